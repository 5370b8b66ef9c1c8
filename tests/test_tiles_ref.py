"""CPU tests of the NumPy TILES codec (tests/tiles_ref.py), the executable
statement of the wire format the GPU encoder and decoder are held to
byte for byte (tests/test_gpu_tiles.py).  Round 4 (ABI 10): a tile's base
bits are stored pixel by pixel (pixel j's low b bits at bit j * b of the
channel's b words)."""
import numpy as np

import tiles_ref as T


def _round_trip(a):
    h, w = a.shape[:2]
    s = T.encode(a)
    d = T.decode(s, w, h)
    assert np.array_equal(d[..., :3].view(np.uint32), a[..., :3].view(np.uint32))
    return s


def test_round_trip_special_values_and_noise():
    rng = np.random.default_rng(7)
    a = rng.standard_normal((19, 29, 3)).astype(np.float32)
    bits = a.view(np.uint32)
    bits[0, :6, 0] = [0x00000000, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00001, 0x00000001]
    bits[3, 4, 1] = 0x80000003            # negative denormal
    bits[5:9, 5:9, 2] = rng.integers(0, 2 ** 32, (4, 4), dtype=np.uint32)   # 32-bit residuals
    _round_trip(a)


def test_wide_tiles_exceed_64_words():
    """Residuals of ~32 bits in all three channels: b0 + b1 + b2 > 64 words,
    the decoder's second batch of words."""
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2 ** 32, (8, 8, 3), dtype=np.uint32).view(np.float32)
    s = _round_trip(a)
    head = np.frombuffer(s[T.head_offset(1):T.data_offset(1)].tobytes(), dtype=np.uint32)
    assert (head[0] & 63) + (head[0] >> 6 & 63) + (head[0] >> 12 & 63) > 64


def test_base_bits_are_lane_major():
    """A tile whose channel-0 gradient residuals are all 3 (pixel 0 travels
    raw): zigzag 6, so b = 3 (cheaper than any escape) and pixel j's bits
    sit at bit 3 j of the channel's 3 words; channels 1 and 2 are constant
    (b = 0)."""
    r = np.full((8, 8), 3, dtype=np.uint64)
    r[0, 0] = 1000
    u = (r.cumsum(axis=0).cumsum(axis=1) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    a = np.zeros((8, 8, 3), dtype=np.float32)
    a[..., 0] = T.ordered(u).view(np.float32)
    a[..., 1] = 1.0
    a[..., 2] = -2.0
    s = _round_trip(a)
    head = np.frombuffer(s[T.head_offset(1):T.data_offset(1)].tobytes(), dtype=np.uint32)
    b = [int(head[0] >> (6 * c) & 63) for c in range(3)]
    assert b == [3, 0, 0] and (head[0] >> 26 & 7) == 0
    words = int.from_bytes(s[T.data_offset(1):T.data_offset(1) + 8 * 3].tobytes(), "little")
    z = [(words >> (3 * j)) & 7 for j in range(64)]
    assert z == [0] + [6] * 63
