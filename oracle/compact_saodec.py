"""TEST INFRASTRUCTURE: merge TAppEncoder_saodec captures (oracle/saodec_capture.cpp) record-wise
into one fixture, with the per-CTU statistics stored as int32 (a 64x64 CTU's counts and
difference sums fit) and the CTUs per slice of each picture appended to meta.
usage: python oracle/compact_saodec.py out.bin slice_ctus1:in1.bin slice_ctus2:in2.bin ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io  # noqa: E402


def main():
    out, specs = sys.argv[1], sys.argv[2:]
    meta, f64, stats, params = [], [], [], []
    for spec in specs:
        sc, path = spec.split(":", 1)
        g = golden_io.load(path)
        m = g["meta"].astype(np.int32)
        meta.append(np.concatenate([m, np.full((m.shape[0], 1), int(sc), np.int32)], axis=1))
        f64.append(g["f64"])
        s = g["stats"]
        assert np.abs(s).max() < 2 ** 31
        stats.append(s.astype(np.int32))
        params.append(g["params"])
    golden_io.save(out, {"meta": np.concatenate(meta), "f64": np.concatenate(f64), "stats": np.concatenate(stats),
                         "params": np.concatenate(params)})


if __name__ == "__main__":
    main()
