"""TEST INFRASTRUCTURE: tests/golden/gop_plans.json from compact CTU captures (oracle/cu_capture.cpp).

Per picture of a closed HM-16.5rc1 encode, in coding order, the slice set-up TEncGOP::compressGOP gave
it (TEncGOP.cpp:1024-1336): POC, slice type, slice QP, the active reference POC lists, collocated_from_l0,
checkLDC, TMVP, MaxNumMergeCand, the collocated picture and its lists, lambda and the cabac_init table.
video_codecs_amd/gop.py reads the structure fields; the rest pins its lambda / list derivation in
tests/test_gop_cpu.py.  Usage: python3 oracle/gop_plans.py out.json kind=capture.bin [kind=capture.bin ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io  # noqa: E402


def plan(path):
    g = golden_io.load(path)
    out = []
    for pi, pf in zip(g["pic_i32"], g["pic_f64"]):
        pi = [int(x) for x in pi]
        out.append({"poc": pi[2], "slice_type": pi[3], "qp": pi[4], "nref": pi[5:7],
                    "ref_poc": [pi[7:11], pi[11:15]], "col_from_l0": pi[23], "check_ldc": pi[25], "tmvp": pi[26],
                    "max_merge": pi[27], "col_poc": pi[28], "col_nref": pi[29:31], "col_ref_poc": [pi[31:35], pi[35:39]],
                    "chroma_qp": pi[39:41], "lambda_motion": pi[43] & 0xffffffff, "cabac_table": pi[44],
                    "col_valid": pi[45], "lambda": float(pf[0])})
    return out


if __name__ == "__main__":
    res = {}
    for a in sys.argv[2:]:
        kind, path = a.split("=", 1)
        res[kind] = plan(path)
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=0)
