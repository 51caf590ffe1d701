"""Synthetic 8-bit 4:2:0 YUV generator (TEST INFRASTRUCTURE and bench input recipe).

Kinds:
  random  -- BASELINE.md section 3: splitmix64 seeded 0x5EED0000 + frame index,
             every sample is the top byte (x >> 56) of the next draw, Y then Cb then Cr.
  smooth  -- moving sinusoid texture + small splitmix64 noise: gives the encoder real
             motion and a realistic coefficient distribution (used for golden capture).
"""
import sys

import numpy as np

MASK = (1 << 64) - 1


def splitmix64_stream(seed: int, n: int) -> np.ndarray:
    """n successive splitmix64 outputs (uint64) from state `seed` (vectorised)."""
    with np.errstate(over="ignore"):
        k = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_frame(w: int, h: int, index: int) -> np.ndarray:
    n = w * h * 3 // 2
    return (splitmix64_stream(0x5EED0000 + index, n) >> np.uint64(56)).astype(np.uint8)


def smooth_frame(w: int, h: int, index: int) -> np.ndarray:
    out = []
    for cw, ch, scale in ((w, h, 1.0), (w // 2, h // 2, 0.5), (w // 2, h // 2, 0.5)):
        y, x = np.mgrid[0:ch, 0:cw].astype(np.float64)
        x = x / scale + 2.0 * index
        y = y / scale - 1.0 * index
        v = 128 + 60 * np.sin(x * 0.11 + y * 0.05) + 40 * np.cos(y * 0.13 - x * 0.03)
        noise = (splitmix64_stream(0x5EED8000 + index * 7 + len(out), cw * ch) >> np.uint64(61)).astype(np.int64) - 4
        out.append(np.clip(np.rint(v) + noise.reshape(ch, cw), 0, 255).astype(np.uint8).ravel())
    return np.concatenate(out)


def _texture_canvas(cw: int, ch: int, seed: int) -> np.ndarray:
    """A static detailed texture: splitmix64 noise box-filtered twice (3x3) plus two sinusoids."""
    n = (splitmix64_stream(seed, cw * ch) >> np.uint64(56)).astype(np.float64).reshape(ch, cw)
    for _ in range(2):
        p = np.pad(n, 1, mode="edge")
        n = sum(p[dy:dy + ch, dx:dx + cw] for dy in range(3) for dx in range(3)) / 9.0
    y, x = np.mgrid[0:ch, 0:cw].astype(np.float64)
    return (n - 128.0) * 2.2 + 128.0 + 30 * np.sin(x * 0.21 + y * 0.07) + 20 * np.cos(y * 0.17 - x * 0.05)


def texture_frame(w: int, h: int, index: int) -> np.ndarray:
    """texture -- a detailed background in global motion (2, -1) per frame, two objects of another
    texture moving on their own paths, per-frame noise of +-4: real uni / bi-prediction choices
    (used for the randomaccess CTU captures)."""
    out = []
    for c, (cw, ch) in enumerate(((w, h), (w // 2, h // 2), (w // 2, h // 2))):
        s = 1 if c == 0 else 2
        pad = 96 // s
        bg = _texture_canvas(cw + 2 * pad, ch + 2 * pad, 0x7E470000 + c)
        ox, oy = pad + (2 * index) // s, pad - index // s
        f = bg[oy:oy + ch, ox:ox + cw].copy()
        obj = _texture_canvas(64 // s, 48 // s, 0x7E471000 + c) * 0.8 + 25
        for k, (x0, y0, vx, vy) in enumerate(((40, 30, 5, 2), (260, 150, -3, -4))):
            ax, ay = (x0 + vx * index) // s, (y0 + vy * index) // s
            oh, ow = obj.shape
            ys, xs = max(ay, 0), max(ax, 0)
            ye, xe = min(ay + oh, ch), min(ax + ow, cw)
            if ye > ys and xe > xs:
                f[ys:ye, xs:xe] = obj[ys - ay:ye - ay, xs - ax:xe - ax] + 12 * k
        noise = (splitmix64_stream(0x7E472000 + index * 7 + c, cw * ch) >> np.uint64(61)).astype(np.int64) - 4
        out.append(np.clip(np.rint(f) + noise.reshape(ch, cw), 0, 255).astype(np.uint8).ravel())
    return np.concatenate(out)


def write_yuv(path: str, kind: str, w: int, h: int, frames: int) -> None:
    gen = {"random": random_frame, "smooth": smooth_frame, "texture": texture_frame}[kind]
    with open(path, "wb") as f:
        for i in range(frames):
            f.write(gen(w, h, i).tobytes())


if __name__ == "__main__":
    kind, w, h, frames, path = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    write_yuv(path, kind, w, h, frames)
