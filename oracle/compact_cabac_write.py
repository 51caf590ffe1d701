"""TEST INFRASTRUCTURE: merge cabac_write captures (oracle/cabac_write_capture.cpp) into one
golden: records concatenated, byte offsets rebased, coefficient rows packed to w*h levels per
record (coef_flat + coef_off), state rows cut to HVX_NUM_CTX bytes.
usage: python oracle/compact_cabac_write.py out.bin in1.bin in2.bin ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io  # noqa: E402

NUM_CTX = 202


def main():
    out, ins = sys.argv[1], [golden_io.load(p) for p in sys.argv[2:]]
    meta = np.concatenate([g["meta"] for g in ins])
    sizes = (meta[:, 0] * meta[:, 1]).astype(np.int64)
    coef = np.concatenate([g["coef"] for g in ins])
    byte_off, base = [np.zeros(1, np.int64)], 0
    for g in ins:
        byte_off.append(g["byte_off"][1:] + base)
        base += int(g["byte_off"][-1])
    res = {
        "meta": meta,
        "coef_flat": np.concatenate([coef[i, :sizes[i]] for i in range(len(meta))]).astype(np.int16),
        "coef_off": np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64),
        "states_before": np.ascontiguousarray(np.concatenate([g["states_before"] for g in ins])[:, :NUM_CTX]),
        "states_after": np.ascontiguousarray(np.concatenate([g["states_after"] for g in ins])[:, :NUM_CTX]),
        "regs": np.concatenate([g["regs"] for g in ins]),
        "bytes": np.concatenate([g["bytes"] for g in ins]),
        "byte_off": np.concatenate(byte_off).astype(np.int64),
    }
    golden_io.save(out, res)


if __name__ == "__main__":
    main()
