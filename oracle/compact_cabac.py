"""TEST INFRASTRUCTURE: pack the coefficient rows of a cabac golden (oracle/cabac_capture.cpp,
1024 int16 per record) into one flat array of w*h levels per record plus offsets, and the
202-model state rows to HVX_NUM_CTX bytes.  usage: python oracle/compact_cabac.py golden.bin"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io  # noqa: E402

NUM_CTX = 202


def main():
    path = sys.argv[1]
    g = golden_io.load(path)
    if "coef" not in g:
        return
    meta = g["meta"]
    sizes = (meta[:, 0] * meta[:, 1]).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    flat = np.concatenate([g["coef"][i, :sizes[i]] for i in range(len(meta))])
    out = {k: v for k, v in g.items() if k not in ("coef", "states_before", "states_after")}
    out["coef_flat"] = flat.astype(np.int16)
    out["coef_off"] = off
    out["states_before"] = np.ascontiguousarray(g["states_before"][:, :NUM_CTX])
    out["states_after"] = np.ascontiguousarray(g["states_after"][:, :NUM_CTX])
    golden_io.save(path, out)


if __name__ == "__main__":
    main()
