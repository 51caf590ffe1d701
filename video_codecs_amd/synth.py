"""Synthetic bench input: splitmix64 seeded 0x5EED0000 + frame index, every
sample the top byte (x >> 56) of the next draw, Y then Cb then Cr (8-bit 4:2:0).  The bench's own
copy of the recipe, so the measured path imports nothing from oracle/ (tests check that the two
generators agree)."""
import numpy as np


def splitmix64_stream(seed, n):
    """n successive splitmix64 outputs (uint64) from state `seed`."""
    with np.errstate(over="ignore"):
        k = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_frame(w, h, index):
    """One w x h 4:2:0 frame, planar Y | Cb | Cr bytes."""
    return (splitmix64_stream(0x5EED0000 + index, w * h * 3 // 2) >> np.uint64(56)).astype(np.uint8)


def random_frame_torch(w, h, index, device="cuda"):
    """random_frame computed with torch int64 arithmetic on `device` (the bench's many closed segments
    make their originals on the GPU): the same splitmix64 stream -- multiplications wrap modulo 2^64,
    the logical right shifts are arithmetic shifts masked to the low bits -- so the bytes are identical
    (tests/test_abi_cpu.py checks them against random_frame)."""
    import torch

    def c(v):  # a uint64 constant as the int64 of the same bits
        return v - (1 << 64) if v >= 1 << 63 else v

    def shr(z, s):
        return (z >> s) & ((1 << (64 - s)) - 1)
    n = w * h * 3 // 2
    k = torch.arange(1, n + 1, dtype=torch.int64, device=device)
    z = c(0x5EED0000 + index) + k * c(0x9E3779B97F4A7C15)
    z = (z ^ shr(z, 30)) * c(0xBF58476D1CE4E5B9)
    z = (z ^ shr(z, 27)) * c(0x94D049BB133111EB)
    z = z ^ shr(z, 31)
    return shr(z, 56).to(torch.uint8)


def luma_plane(w, h, index, margin=80):
    """The frame's luma as an 8-bit padded plane (HVX_PLANE_MARGIN border, edges replicated)."""
    y = random_frame(w, h, index)[: w * h].reshape(h, w)
    return np.pad(y, margin, mode="edge")


def yuv_planes(w, h, index, margin=80):
    """The frame as three 8-bit padded planes (Y with margin, Cb / Cr with margin // 2, edges replicated)."""
    f = random_frame(w, h, index)
    n, c = w * h, (w // 2) * (h // 2)
    y = f[:n].reshape(h, w)
    cb = f[n:n + c].reshape(h // 2, w // 2)
    cr = f[n + c:n + 2 * c].reshape(h // 2, w // 2)
    return np.pad(y, margin, mode="edge"), np.pad(cb, margin // 2, mode="edge"), np.pad(cr, margin // 2, mode="edge")
