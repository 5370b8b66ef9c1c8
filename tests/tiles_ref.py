"""NumPy reference of the TILES wire format (include/sdf_abi.h, SDF_FORMAT_TILES).

TEST INFRASTRUCTURE: the executable statement of the stream layout that the
HIP encoder (render_kernel.inc store_tiles + tiles.hip compaction) and decoder
(tiles.hip decode_tiles) must agree with.  The tests use it as a checker:
GPU streams are compared byte for byte with encode() (plane blocks are in tile
order on both sides) and decoded with decode(); encode() streams feed the GPU
decoder.  Never on the product path.
"""
from __future__ import annotations

import numpy as np

MAX_PLANES = 3 * 32


def tiles_shape(width: int, rows: int) -> tuple[int, int]:
    return (rows + 7) // 8, (width + 7) // 8


def head_offset(ntiles: int) -> int:
    return (8 + 4 * ntiles + 15) // 16 * 16


def data_offset(ntiles: int) -> int:
    return head_offset(ntiles) + 16 * ntiles


def capacity(width: int, rows: int) -> int:
    """Worst-case stream size (all residuals 32 bits wide)."""
    ty, tx = tiles_shape(width, rows)
    n = ty * tx
    return data_offset(n) + 8 * MAX_PLANES * n


def ordered(bits: np.ndarray) -> np.ndarray:
    """float bits -> ordered integer (an involution: also the inverse)."""
    bits = bits.astype(np.uint32)
    return np.where(bits & 0x80000000, bits ^ np.uint32(0x7FFFFFFF), bits).astype(np.uint32)


def _tiles(a: np.ndarray, rows: int, width: int) -> np.ndarray:
    """[rows, width] -> [ntiles, 8, 8] with zero padding outside the frame."""
    ty, tx = tiles_shape(width, rows)
    p = np.zeros((ty * 8, tx * 8), dtype=a.dtype)
    p[:rows, :width] = a
    return p.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 8, 8)


def _bit_length(m: np.ndarray) -> np.ndarray:
    w = np.zeros(m.shape, dtype=np.int64)
    v = m.astype(np.uint64).copy()
    while np.any(v):
        nz = v != 0
        w += nz
        v >>= np.uint64(1)
    return w


def encode(rgb: np.ndarray) -> np.ndarray:
    """[rows, width, >=3] float32 -> uint8 stream."""
    rows, width = rgb.shape[:2]
    ty, tx = tiles_shape(width, rows)
    n = ty * tx
    inside = _tiles(np.ones((rows, width), dtype=np.uint8), rows, width).reshape(n, 64) == 1
    heads = np.zeros((n, 4), dtype=np.uint32)
    planes_c, widths = [], []
    bitpos = np.arange(64, dtype=np.uint64)
    for c in range(3):
        u = ordered(np.ascontiguousarray(rgb[..., c], dtype=np.float32).view(np.uint32))
        t = _tiles(u, rows, width).astype(np.uint64)
        L = np.zeros_like(t); L[:, :, 1:] = t[:, :, :-1]
        U = np.zeros_like(t); U[:, 1:, :] = t[:, :-1, :]
        UL = np.zeros_like(t); UL[:, 1:, 1:] = t[:, :-1, :-1]
        r = ((t - L - U + UL) & np.uint64(0xFFFFFFFF)).astype(np.int64)   # mod 2^32
        r = np.where(r >= 2 ** 31, r - 2 ** 32, r)
        z = np.where(r >= 0, 2 * r, -2 * r - 1).astype(np.uint64).reshape(n, 64)
        heads[:, 1 + c] = t.reshape(n, 64)[:, 0].astype(np.uint32)
        z[:, 0] = 0
        z[~inside] = 0
        w = _bit_length(z.max(axis=1))
        planes = np.zeros((n, 32), dtype=np.uint64)
        for b in range(32):
            bits = (z >> np.uint64(b)) & np.uint64(1)
            planes[:, b] = (bits << bitpos).sum(axis=1, dtype=np.uint64)
        planes_c.append(planes)
        widths.append(w)
    heads[:, 0] = (widths[0] | widths[1] << 8 | widths[2] << 16).astype(np.uint32)
    table = np.zeros(n, dtype=np.uint32)
    blocks, off = [], 0
    for i in range(n):
        blk = np.concatenate([planes_c[c][i, :widths[c][i]] for c in range(3)])
        table[i] = off
        blocks.append(blk.tobytes())
        off += 8 * blk.size
    out = np.zeros(data_offset(n) + off, dtype=np.uint8)
    out[:8] = np.frombuffer(np.array([off, n], dtype=np.uint32).tobytes(), dtype=np.uint8)
    out[8:8 + 4 * n] = np.frombuffer(table.tobytes(), dtype=np.uint8)
    out[head_offset(n):data_offset(n)] = np.frombuffer(heads.tobytes(), dtype=np.uint8)
    out[data_offset(n):] = np.frombuffer(b"".join(blocks), dtype=np.uint8)
    return out


def decode(stream: np.ndarray, width: int, rows: int) -> np.ndarray:
    """uint8 stream -> [rows, width, 4] float32, alpha = 1."""
    s = np.asarray(stream, dtype=np.uint8)
    ty, tx = tiles_shape(width, rows)
    n = ty * tx
    used, ntiles = np.frombuffer(s[:8].tobytes(), dtype=np.uint32)
    if ntiles != n:
        raise ValueError(f"stream has {ntiles} tiles, expected {n}")
    table = np.frombuffer(s[8:8 + 4 * n].tobytes(), dtype=np.uint32)
    heads = np.frombuffer(s[head_offset(n):data_offset(n)].tobytes(), dtype=np.uint32).reshape(n, 4)
    base = data_offset(n)
    out = np.ones((ty * 8, tx * 8, 4), dtype=np.float32)
    bitpos = np.arange(64, dtype=np.uint64)
    for i in range(n):
        ws = [int(heads[i, 0]) & 255, int(heads[i, 0]) >> 8 & 255, int(heads[i, 0]) >> 16 & 255]
        k = base + int(table[i])
        if int(table[i]) + 8 * sum(ws) > used:
            raise ValueError("planes beyond the used bytes")
        yi, xi = divmod(i, tx)
        for c in range(3):
            planes = np.frombuffer(s[k:k + 8 * ws[c]].tobytes(), dtype=np.uint64)
            k += 8 * ws[c]
            z = np.zeros(64, dtype=np.uint64)
            for b, p in enumerate(planes):
                z |= ((p >> bitpos) & np.uint64(1)) << np.uint64(b)
            zi = z.astype(np.int64)
            r = np.where(zi & 1, -(zi >> 1) - 1, zi >> 1)             # unzigzag
            r = (r & 0xFFFFFFFF).astype(np.uint64)
            r[0] = int(heads[i, 1 + c])
            u = r.reshape(8, 8).cumsum(axis=0).cumsum(axis=1) & np.uint64(0xFFFFFFFF)
            bits = ordered(u.astype(np.uint32))
            out[yi * 8:yi * 8 + 8, xi * 8:xi * 8 + 8, c] = bits.view(np.float32)
    return out[:rows, :width]


def stream_bytes(stream: np.ndarray) -> int:
    """The meaningful prefix of a stream: tables plus used plane bytes."""
    used, n = np.frombuffer(np.asarray(stream[:8], dtype=np.uint8).tobytes(), dtype=np.uint32)
    return data_offset(int(n)) + int(used)
