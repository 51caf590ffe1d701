"""Debugging aid: decide the captured CTUs with a libhvx build selected by HVX_LIB_PATH (e.g. an
HM_CHECKS build) and print the first failed engine check per job (State.dbg: code, a, b) and the
first mismatches against the reference.  python -m tests.hm_debug [capture] [mode] [pics] [serial]"""
import sys

import numpy as np

from tests import hm_cases


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ctu_ldp_rand.bin"
    mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    pics = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
    serial = len(sys.argv) > 4 and sys.argv[4] == "serial"
    g, plan, out = hm_cases.run_capture(name, mode, pics, serial=serial)
    dbg = hm_cases.LAST_ENGINE[0].last_debug
    bad_jobs = np.flatnonzero(dbg[:, 0])
    print("%s mode %d: %d jobs, %d with a failed check" % (name, mode, len(dbg), len(bad_jobs)))
    codes = {}
    for j in bad_jobs:
        codes.setdefault(int(dbg[j, 0]), []).append((int(j), int(dbg[j, 1]), int(dbg[j, 2])))
    for c, lst in sorted(codes.items()):
        print("  check %d: %d jobs, first %s" % (c, len(lst), lst[:4]))
    bad = hm_cases.compare(g, plan, out)
    print("%d mismatching CTUs; first: %s" % (len(bad), bad[:4]))


if __name__ == "__main__":
    main()
