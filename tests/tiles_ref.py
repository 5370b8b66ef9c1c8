"""NumPy reference of the TILES wire format (include/sdf_abi.h, SDF_FORMAT_TILES).

TEST INFRASTRUCTURE: the executable statement of the stream layout that the
HIP encoder (render_kernel.inc store_tiles + tiles.hip compaction) and decoder
(tiles.hip decode_tiles) must agree with.  The tests use it as a checker:
GPU streams are compared byte for byte with encode() (plane blocks are in tile
order on both sides) and decoded with decode(); encode() streams feed the GPU
decoder.  Never on the product path.

A stream's three channels hold RGB (header shade mode 0) or, in a stream
rendered by sdf_render, the pixels' shading terms (ao, dif, x; mode 1 fast /
2 exact precision) with the frame's shading constants in the header, from
which the GPU decoder makes the colour (sdf3d_amd/csrc/shade.h).  This module
handles the codec: decode() returns the channel values themselves.
"""
from __future__ import annotations

import numpy as np

MAX_PLANES = 3 * 32
HEADER_BYTES = 64
SHADE_RAW, SHADE_FAST, SHADE_EXACT = 0, 1, 2


def tiles_shape(width: int, rows: int) -> tuple[int, int]:
    return (rows + 7) // 8, (width + 7) // 8


def head_offset(ntiles: int) -> int:
    return (HEADER_BYTES + 4 * ntiles + 15) // 16 * 16


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


# Per channel the tile keeps the low `b` bits of every residual -- b words,
# pixel j's bits at bit j * b (lane-major, round 4; bit planes before) -- and, when
# some residuals are wider (the tile's widest has `w` bits), an escape for
# them: the 64-bit mask M of those pixels, a width byte w - b, and their
# bits b..w-1 as (w - b)-bit fields.  b is the cheapest of w, w-1, ...,
# w - ESCAPE_WINDOW (>= 0) in bits: 64 b, plus 64 + 8 + (w - b) n with n
# outliers; ties keep the larger b.  The fields are ordered pixel-major:
# pixel by pixel, each pixel's fields of the escaped channels it is an
# outlier of, in channel order -- so pixel j's fields start at bit
# 8 P + sum_c (w_c - b_c) * |{outliers of c below j}|.
ESCAPE_WINDOW = 12


def _choose_base(bl: np.ndarray) -> np.ndarray:
    """[n, 64] bit lengths -> [n] base widths b."""
    w = bl.max(axis=1)
    best_b, best = w.copy(), 64 * w
    for d in range(1, ESCAPE_WINDOW + 1):
        b = w - d
        n = (bl > np.maximum(b, 0)[:, None]).sum(axis=1)
        cost = 64 * np.maximum(b, 0) + 72 + d * n
        take = (b >= 0) & (cost < best)
        best = np.where(take, cost, best)
        best_b = np.where(take, b, best_b)
    return best_b


def _pack_fields(fields) -> bytes:
    """[(value, nbits)] -> little-endian bitstream padded to whole qwords."""
    acc, nbits = 0, 0
    for v, k in fields:
        acc |= (int(v) & ((1 << k) - 1)) << nbits
        nbits += k
    nq = (nbits + 63) // 64
    return acc.to_bytes(8 * nq, "little")


def shade_header(light, material, precision_exact: bool) -> tuple[int, np.ndarray]:
    """(mode, 10 float32 shading constants) a render of this light and
    material writes into its stream header: light.ambient * material.amb[c]
    rounded to fp32, material.dif, material.ref, shininess."""
    la = np.float32(light.ambient)
    k = [np.float32(la * np.float32(material.amb[c])) for c in range(3)]
    k += [np.float32(material.dif[c]) for c in range(3)]
    k += [np.float32(material.ref[c]) for c in range(3)]
    k.append(np.float32(material.shininess))
    return (SHADE_EXACT if precision_exact else SHADE_FAST), np.array(k, dtype=np.float32)


def header(stream: np.ndarray) -> dict:
    """The stream header's fields."""
    w = np.frombuffer(np.asarray(stream[:HEADER_BYTES], dtype=np.uint8).tobytes(), dtype=np.uint32)
    return {"used": int(w[0]), "ntiles": int(w[1]), "shade": int(w[2]),
            "k": w[4:14].view(np.float32).copy()}


def encode(rgb: np.ndarray, shade: tuple[int, np.ndarray] | None = None) -> np.ndarray:
    """[rows, width, >=3] float32 -> uint8 stream; `shade` = (mode, constants)
    for a stream of shading terms (shade_header), None for RGB."""
    rows, width = rgb.shape[:2]
    ty, tx = tiles_shape(width, rows)
    n = ty * tx
    inside = _tiles(np.ones((rows, width), dtype=np.uint8), rows, width).reshape(n, 64) == 1
    heads = np.zeros((n, 4), dtype=np.uint32)
    zs, bls, bases = [], [], []
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
        bl = _bit_length(z)
        zs.append(z)
        bls.append(bl)
        bases.append(_choose_base(bl))
    table = np.zeros(n, dtype=np.uint32)
    blocks, off = [], 0
    for i in range(n):
        base_planes, masks, deltas, fields = [], [], [], []
        present = 0
        outl = []
        for c in range(3):
            z, b = zs[c][i], int(bases[c][i])
            w = int(bls[c][i].max())
            # lane-major: pixel j's low b bits at bit j * b of the channel's
            # b words
            low = z & np.uint64((1 << b) - 1) if b else np.zeros(64, dtype=np.uint64)
            acc = 0
            for j in range(64 if b else 0):
                acc |= int(low[j]) << (j * b)
            base_planes.extend(int(acc >> (64 * p)) & 0xFFFFFFFFFFFFFFFF for p in range(b))
            if b < w:
                present |= 1 << c
                o = bls[c][i] > b
                outl.append((c, b, w - b, o))
                masks.append(int(sum(1 << int(j) for j in np.nonzero(o)[0])))
                deltas.append((w - b, 8))
        for j in range(64):
            for c, b, d, o in outl:
                if o[j]:
                    fields.append((int(zs[c][i][j]) >> b, d))
        data = (np.array(base_planes + masks, dtype=np.uint64).tobytes()
                + _pack_fields(deltas + fields))
        nq = len(data) // 8
        heads[i, 0] = (int(bases[0][i]) | int(bases[1][i]) << 6 | int(bases[2][i]) << 12
                       | nq << 18 | present << 26)
        table[i] = off
        blocks.append(data)
        off += len(data)
    out = np.zeros(data_offset(n) + off, dtype=np.uint8)
    hw = np.zeros(HEADER_BYTES // 4, dtype=np.uint32)
    hw[0], hw[1] = off, n
    if shade is not None:
        hw[2] = shade[0]
        hw[4:14] = np.asarray(shade[1], dtype=np.float32).view(np.uint32)
    out[:HEADER_BYTES] = np.frombuffer(hw.tobytes(), dtype=np.uint8)
    out[HEADER_BYTES:HEADER_BYTES + 4 * n] = np.frombuffer(table.tobytes(), dtype=np.uint8)
    out[head_offset(n):data_offset(n)] = np.frombuffer(heads.tobytes(), dtype=np.uint8)
    out[data_offset(n):] = np.frombuffer(b"".join(blocks), dtype=np.uint8)
    return out


def decode(stream: np.ndarray, width: int, rows: int) -> np.ndarray:
    """uint8 stream -> [rows, width, 4] float32: the three channel values
    (RGB, or the shading terms of a rendered stream), alpha = 1."""
    s = np.asarray(stream, dtype=np.uint8)
    ty, tx = tiles_shape(width, rows)
    n = ty * tx
    used, ntiles = np.frombuffer(s[:8].tobytes(), dtype=np.uint32)
    if ntiles != n:
        raise ValueError(f"stream has {ntiles} tiles, expected {n}")
    table = np.frombuffer(s[HEADER_BYTES:HEADER_BYTES + 4 * n].tobytes(), dtype=np.uint32)
    heads = np.frombuffer(s[head_offset(n):data_offset(n)].tobytes(), dtype=np.uint32).reshape(n, 4)
    base = data_offset(n)
    out = np.ones((ty * 8, tx * 8, 4), dtype=np.float32)
    for i in range(n):
        h = int(heads[i, 0])
        bs = [h & 63, h >> 6 & 63, h >> 12 & 63]
        nq, present = h >> 18 & 255, h >> 26 & 7
        if int(table[i]) + 8 * nq > used:
            raise ValueError("tile data beyond the used bytes")
        k = base + int(table[i])
        q = np.frombuffer(s[k:k + 8 * nq].tobytes(), dtype=np.uint64)
        pc = [c for c in range(3) if present >> c & 1]
        B, P = sum(bs), len(pc)
        bits = int.from_bytes(q[B + P:].tobytes(), "little")
        deltas = {c: bits >> (8 * j) & 255 for j, c in enumerate(pc)}
        masks = {c: int(q[B + j]) for j, c in enumerate(pc)}
        zs = []
        kp = 0
        for c in range(3):
            b = bs[c]
            acc = int.from_bytes(q[kp:kp + b].tobytes(), "little")
            z = np.array([acc >> (j * b) & ((1 << b) - 1) for j in range(64)], dtype=np.uint64)
            kp += b
            zs.append(z)
        pos = 8 * P
        for j in range(64):
            for c in pc:
                if masks[c] >> j & 1:
                    d = deltas[c]
                    zs[c][j] |= np.uint64((bits >> pos & ((1 << d) - 1)) << bs[c])
                    pos += d
        yi, xi = divmod(i, tx)
        for c in range(3):
            z = zs[c]
            zi = z.astype(np.int64)
            r = np.where(zi & 1, -(zi >> 1) - 1, zi >> 1)             # unzigzag
            r = (r & 0xFFFFFFFF).astype(np.uint64)
            r[0] = int(heads[i, 1 + c])
            u = r.reshape(8, 8).cumsum(axis=0).cumsum(axis=1) & np.uint64(0xFFFFFFFF)
            fb = ordered(u.astype(np.uint32))
            out[yi * 8:yi * 8 + 8, xi * 8:xi * 8 + 8, c] = fb.view(np.float32)
    return out[:rows, :width]


def stream_bytes(stream: np.ndarray) -> int:
    """The meaningful prefix of a stream: tables plus used plane bytes."""
    used, n = np.frombuffer(np.asarray(stream[:8], dtype=np.uint8).tobytes(), dtype=np.uint32)
    return data_offset(int(n)) + int(used)
