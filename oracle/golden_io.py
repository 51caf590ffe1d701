"""Reader for the "HVXG" golden containers in tests/golden/ (writer: oracle/golden_writer.h).

TEST INFRASTRUCTURE.  Pure numpy, no pickle.
"""
import struct

import numpy as np

_DT = {"u8": np.uint8, "i8": np.int8, "i16": np.int16, "i32": np.int32, "u32": np.uint32, "i64": np.int64,
       "f32": np.float32, "f64": np.float64}


def load(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"HVXG":
        raise ValueError(f"{path}: not an HVXG golden file")
    (n,) = struct.unpack_from("<I", data, 4)
    off = 8
    for _ in range(n):
        name = data[off:off + 32].split(b"\0", 1)[0].decode()
        dt = data[off + 32:off + 40].split(b"\0", 1)[0].decode()
        nd, s0, s1, s2, s3 = struct.unpack_from("<5I", data, off + 40)
        off += 60
        shape = (s0, s1, s2, s3)[:nd]
        dtype = np.dtype(_DT[dt])
        count = int(np.prod(shape)) if nd else 1
        out[name] = np.frombuffer(data, dtype=dtype, count=count, offset=off).reshape(shape).copy()
        off += count * dtype.itemsize
    return out


_NAME = {np.dtype(v): k for k, v in _DT.items()}


def save(path, arrays):
    """Write {name: ndarray} (<= 4 dims) as an HVXG container (same layout as golden_writer.h)."""
    parts = [b"HVXG", struct.pack("<I", len(arrays))]
    for name, a in arrays.items():
        a = np.ascontiguousarray(a)
        shape = list(a.shape) + [0] * (4 - a.ndim)
        parts.append(name.encode().ljust(32, b"\0") + _NAME[a.dtype].encode().ljust(8, b"\0"))
        parts.append(struct.pack("<5I", a.ndim, *shape))
        parts.append(a.tobytes())
    with open(path, "wb") as f:
        f.write(b"".join(parts))
