"""TEST INFRASTRUCTURE: concatenate HVXG golden containers record-wise (axis 0).
Arrays named in SHARED must be identical in every input and are kept once.
usage: python oracle/merge_goldens.py out.bin in1.bin in2.bin ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io  # noqa: E402

SHARED = {"entropy_bits"}


def main():
    out, ins = sys.argv[1], [golden_io.load(p) for p in sys.argv[2:]]
    merged = {}
    for k in ins[0]:
        if k in SHARED:
            for g in ins[1:]:
                assert np.array_equal(g[k], ins[0][k]), k
            merged[k] = ins[0][k]
        else:
            merged[k] = np.concatenate([g[k] for g in ins])
    golden_io.save(out, merged)


if __name__ == "__main__":
    main()
