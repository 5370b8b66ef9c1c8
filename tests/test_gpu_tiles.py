"""GPU tests of the TILES wire format (include/sdf_abi.h SDF_FORMAT_TILES).

The multi-device gather ships each rank's rows as a lossless compressed
stream written by the render kernel itself; rank 0 decodes it straight into
the assembled RGBA32F frame.  Lossless is the whole contract, so every test is
bit-exact: the decoded frame must equal the RGBA32F render byte for byte.
The format is pinned against the NumPy restatement in tests/tiles_ref.py in
both directions (GPU stream -> NumPy decoder, NumPy stream -> GPU decoder).
A rendered stream carries the pixels' shading terms (SDF_FORMAT_SHADE32F),
from which the decoder makes the colour: bit-identical to the render's own.
"""
import numpy as np
import pytest

import tiles_ref
from sdf3d_amd import abi, renderer as R, scenes

pytestmark = pytest.mark.gpu

CASES = [("REF", 37, 23, 0), ("C3", 64, 64, 1), ("C3", 320, 180, 2), ("C5", 96, 72, 0),
         ("C1", 9, 200, 0), ("C2", 200, 9, 3)]


def frame(cfg, w, h, pose, prec, fmt):
    f = scenes.config(cfg, w, h, precision=prec, pose=pose)
    f.params.output_format = fmt
    return f


def render_pair(rd, cfg, w, h, pose, prec, t=None):
    import torch
    ref, _ = rd.render(frame(cfg, w, h, pose, prec, abi.FORMAT_RGBA32F), t)
    st, _ = rd.render(frame(cfg, w, h, pose, prec, abi.FORMAT_TILES), t)
    torch.cuda.synchronize()
    return ref, st


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                          np.ascontiguousarray(b).view(np.uint32))


@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
@pytest.mark.parametrize("cfg,w,h,pose", CASES)
def test_tiles_round_trip_bit_exact(renderer, cfg, w, h, pose, prec):
    import torch
    ref, st = render_pair(renderer, cfg, w, h, pose, prec)
    out = renderer.tiles_decode(st, 1, st.numel(), w, h)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), ref.cpu().numpy())
    n = R.tiles_stream_bytes(st)
    assert n <= st.numel()


def shade_terms(rd, cfg, w, h, pose, prec, t=None):
    import torch
    sh, _ = rd.render(frame(cfg, w, h, pose, prec, abi.FORMAT_SHADE32F), t)
    torch.cuda.synchronize()
    return sh.cpu().numpy()


@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
@pytest.mark.parametrize("cfg,w,h,pose", CASES[:4])
def test_gpu_stream_decodes_with_reference(renderer, cfg, w, h, pose, prec):
    """The stream the kernel writes is the documented layout: byte for byte
    the NumPy encoder's stream of the frame's shading terms (SHADE32F) with
    the frame's shading header, and the NumPy decoder reads the terms back to
    the same bits."""
    _, st = render_pair(renderer, cfg, w, h, pose, prec)
    s = st.cpu().numpy()
    s = s[:tiles_ref.stream_bytes(s)]
    assert R.tiles_stream_bytes(st) == s.size
    terms = shade_terms(renderer, cfg, w, h, pose, prec)
    f = frame(cfg, w, h, pose, prec, abi.FORMAT_TILES)
    hdr = tiles_ref.shade_header(f.light, f.material, prec == abi.PRECISION_EXACT)
    e = tiles_ref.encode(terms, hdr)
    n = tiles_ref.tiles_shape(w, h)[0] * tiles_ref.tiles_shape(w, h)[1]
    table_end, head = tiles_ref.HEADER_BYTES + 4 * n, tiles_ref.head_offset(n)
    assert s.size == e.size
    # every defined field (the alignment gap after the offset table is not)
    assert np.array_equal(s[:table_end], e[:table_end])
    assert np.array_equal(s[head:], e[head:])
    assert tiles_ref.header(s)["shade"] == hdr[0]
    assert same_bits(tiles_ref.decode(s, w, h)[..., :3], terms[..., :3])


@pytest.mark.parametrize("cfg,w,h,pose", CASES[:4])
def test_reference_stream_decodes_on_gpu(renderer, cfg, w, h, pose):
    """The GPU decoder reads streams written by the NumPy encoder: RGB
    streams (header mode 0) to their values, shading-term streams to the
    render's own colours."""
    import torch
    ref, _ = render_pair(renderer, cfg, w, h, pose, abi.PRECISION_FAST)
    host = ref.cpu().numpy()
    buf = torch.zeros(tiles_ref.capacity(w, h), dtype=torch.uint8, device=renderer.device)
    s = tiles_ref.encode(host)
    buf[:s.size] = torch.from_numpy(s).to(renderer.device)
    out = renderer.tiles_decode(buf, 1, buf.numel(), w, h)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), host)
    for prec in (abi.PRECISION_FAST, abi.PRECISION_EXACT):
        f = frame(cfg, w, h, pose, prec, abi.FORMAT_RGBA32F)
        want, _ = renderer.render(f)
        terms = shade_terms(renderer, cfg, w, h, pose, prec)
        s = tiles_ref.encode(terms, tiles_ref.shade_header(f.light, f.material,
                                                           prec == abi.PRECISION_EXACT))
        buf.zero_()
        buf[:s.size] = torch.from_numpy(s).to(renderer.device)
        out = renderer.tiles_decode(buf, 1, buf.numel(), w, h)
        torch.cuda.synchronize()
        assert same_bits(out.cpu().numpy(), want.cpu().numpy())


@pytest.mark.parametrize("cfg,w,h,pose", CASES)
def test_exact_terms_equal_oracle_terms(renderer, cfg, w, h, pose):
    """SDF_FORMAT_SHADE32F in exact precision is the oracle's own terms bit
    for bit (oracle.render_terms; their colour is the oracle's colour,
    tests/test_terms.py)."""
    import oracle
    terms = shade_terms(renderer, cfg, w, h, pose, abi.PRECISION_EXACT)
    f = frame(cfg, w, h, pose, abi.PRECISION_EXACT, abi.FORMAT_SHADE32F)
    ref = oracle.render_terms(f)
    assert same_bits(terms, ref)


@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
def test_shading_terms_without_ao_or_shadow(renderer, prec):
    """ao is 1 without AO (the colour's la * amb * 1 is la * amb bit for
    bit), dif carries no shadow factor without shadows, and the decoded frame
    still equals the render's."""
    import torch
    w, h = 72, 40
    for flags in (0, abi.FLAG_SHADOW, abi.FLAG_AO):
        f = frame("C3", w, h, 1, prec, abi.FORMAT_RGBA32F)
        f.params.flags = flags
        want, _ = renderer.render(f)
        fs = f.copy()
        fs.params.output_format = abi.FORMAT_SHADE32F
        terms, _ = renderer.render(fs)
        ft = f.copy()
        ft.params.output_format = abi.FORMAT_TILES
        st, _ = renderer.render(ft)
        out = renderer.tiles_decode(st, 1, st.numel(), w, h)
        torch.cuda.synchronize()
        assert same_bits(out.cpu().numpy(), want.cpu().numpy())
        tm = terms.cpu().numpy()
        if not flags & abi.FLAG_AO:
            assert np.all(tm[..., 0] == 1.0)
        assert np.all(tm[..., 3] == 1.0)


def test_special_values_round_trip(renderer):
    """NaN payloads, infinities, -0 and negative values survive the reference
    encoder -> GPU decoder path bit for bit (the ordered map is an involution
    and the residual arithmetic is mod 2^32)."""
    import torch
    rng = np.random.default_rng(5)
    w, h = 29, 17
    a = rng.standard_normal((h, w, 4)).astype(np.float32)
    bits = a.view(np.uint32)
    bits.flat[::7] = 0x7FC00123
    bits.flat[::11] = 0x80000000
    bits.flat[::13] = 0xFF800000
    a[..., 3] = 1.0
    s = tiles_ref.encode(a)
    buf = torch.zeros(tiles_ref.capacity(w, h), dtype=torch.uint8, device=renderer.device)
    buf[:s.size] = torch.from_numpy(s).to(renderer.device)
    out = renderer.tiles_decode(buf, 1, buf.numel(), w, h)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), a)


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("h", [64, 71, 180])
def test_multipart_decode_assembles_frame(renderer, world, h):
    """Each rank's TILES stream of tiling {8, r, world}, decoded together,
    is the whole-frame RGBA32F render (decode fused with the de-interleave)."""
    import torch
    w = 96
    whole, _ = renderer.render(frame("C3", w, h, 1, abi.PRECISION_FAST, abi.FORMAT_RGBA32F))
    stride = R.tiles_bytes(w, R.owned_rows(h, R.tiling(0, world, 8)))
    parts = torch.zeros(world * stride, dtype=torch.uint8, device=renderer.device)
    for r in range(world):
        t = R.tiling(r, world, 8)
        if R.owned_rows(h, t) == 0:
            continue
        f = frame("C3", w, h, 1, abi.PRECISION_FAST, abi.FORMAT_TILES)
        renderer.render(f, t, out=parts[r * stride:(r + 1) * stride])
    out = renderer.tiles_decode(parts, world, stride, w, h, 8)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), whole.cpu().numpy())


def test_steps_unchanged_by_tiles_output(renderer):
    import torch
    f32 = frame("C3", 64, 40, 2, abi.PRECISION_FAST, abi.FORMAT_RGBA32F)
    ft = frame("C3", 64, 40, 2, abi.PRECISION_FAST, abi.FORMAT_TILES)
    _, s1 = renderer.render(f32, steps=True)
    _, s2 = renderer.render(ft, steps=True)
    torch.cuda.synchronize()
    assert torch.equal(s1, s2)


def test_compression_on_the_bench_scene(renderer):
    """The point of the format: the 4K CSG frame (C4, here one 8-row band in
    eight) ships in under a quarter of the bytes of RGB32F (about 2.3 bytes
    per pixel as shading terms; 3.2 as the colour itself, round 2)."""
    import torch
    w, h = 3840, 2160
    t = R.tiling(3, 8, 8)
    f = frame("C4", w, h, 0, abi.PRECISION_FAST, abi.FORMAT_TILES)
    st, _ = renderer.render(f, t)
    torch.cuda.synchronize()
    px = R.owned_rows(h, t) * w
    bpp = R.tiles_stream_bytes(st) / px
    print("C4 TILES bytes/pixel", round(bpp, 3))
    assert bpp < 3.0


@pytest.mark.parametrize("world,shares", [(2, (1, 2)), (3, (2, 3)), (8, (1, 3))])
def test_weighted_tiles_decode_assembles_frame(renderer, world, shares):
    """The frame driver's unequal shares: rank 0 renders its run of blocks in
    place (SDF_TILING_FRAME_ROWS, its part left empty), ranks >= 1 their
    runs as TILES streams; sdf_tiles_decode_tilings puts every row back."""
    import torch
    w, h = 88, 197
    f = frame("C3", w, h, 3, abi.PRECISION_FAST, abi.FORMAT_RGBA32F)
    whole, _ = renderer.render(f)
    tilings = [R.tiling(r, world, 8, shares=shares) for r in range(world)]
    stride = max(R.tiles_bytes(w, R.owned_rows(h, t)) for t in tilings)
    out = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device=renderer.device)
    renderer.render(f, R.tiling(0, world, 8, frame_rows=True, shares=shares), out=out)
    parts = torch.zeros(world * stride, dtype=torch.uint8, device=renderer.device)
    ft = frame("C3", w, h, 3, abi.PRECISION_FAST, abi.FORMAT_TILES)
    for r in range(1, world):
        if R.owned_rows(h, tilings[r]):
            renderer.render(ft, tilings[r], out=parts[r * stride:(r + 1) * stride])
    renderer.tiles_decode(parts, world, stride, w, h, out=out, tilings=tilings)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), whole.cpu().numpy())


@pytest.mark.parametrize("world", [2, 3, 8])
def test_frame_rows_tiling_assembles_in_place(renderer, world):
    """SDF_TILING_FRAME_ROWS: every rank's rows written at their frame
    positions of one buffer equal the whole-frame render; a TILES decode
    skips a part whose header says ntiles = 0 (rank 0's rows rendered in
    place, as the frame driver does)."""
    import torch
    w, h = 80, 71
    f = frame("C3", w, h, 2, abi.PRECISION_FAST, abi.FORMAT_RGBA32F)
    whole, _ = renderer.render(f)
    out = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device=renderer.device)
    for r in range(world):
        renderer.render(f, R.tiling(r, world, 8, frame_rows=True), out=out)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), whole.cpu().numpy())
    # rank 0 in place, ranks 1.. as TILES streams
    out2 = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device=renderer.device)
    renderer.render(f, R.tiling(0, world, 8, frame_rows=True), out=out2)
    stride = R.tiles_bytes(w, R.owned_rows(h, R.tiling(0, world, 8)))
    parts = torch.zeros(world * stride, dtype=torch.uint8, device=renderer.device)
    ft = frame("C3", w, h, 2, abi.PRECISION_FAST, abi.FORMAT_TILES)
    for r in range(1, world):
        if R.owned_rows(h, R.tiling(r, world, 8)):
            renderer.render(ft, R.tiling(r, world, 8), out=parts[r * stride:(r + 1) * stride])
    renderer.tiles_decode(parts, world, stride, w, h, 8, out=out2)
    torch.cuda.synchronize()
    assert same_bits(out2.cpu().numpy(), whole.cpu().numpy())


def _tile_widths(terms):
    """Per tile and channel the widest zigzag residual's bit count (the
    encoder's w), restated with tests/tiles_ref.py's steps."""
    rows, width = terms.shape[:2]
    ty, tx = tiles_ref.tiles_shape(width, rows)
    ws = []
    for c in range(3):
        u = tiles_ref.ordered(np.ascontiguousarray(terms[..., c]).view(np.uint32))
        t = tiles_ref._tiles(u, rows, width).astype(np.uint64)
        L = np.zeros_like(t); L[:, :, 1:] = t[:, :, :-1]
        U = np.zeros_like(t); U[:, 1:, :] = t[:, :-1, :]
        UL = np.zeros_like(t); UL[:, 1:, 1:] = t[:, :-1, :-1]
        r = ((t - L - U + UL) & np.uint64(0xFFFFFFFF)).astype(np.int64)
        r = np.where(r >= 2 ** 31, r - 2 ** 32, r)
        z = np.where(r >= 0, 2 * r, -2 * r - 1).astype(np.uint64).reshape(ty * tx, 64)
        z[:, 0] = 0
        ws.append(tiles_ref._bit_length(z.max(axis=1)))
    return ws


@pytest.mark.parametrize("cfg,w,h,pose", [("C4", 480, 272, 0), ("C5", 320, 200, 0)])
def test_encoder_narrow_and_wide_tiles(renderer, cfg, w, h, pose):
    """The encoder's two paths (render_kernel.inc store_tiles, round 4): a
    tile whose channels 0 and 2 fit 16 bits takes one transpose and one
    base-width search, any other tile two of each.  Frames holding both
    kinds encode byte for byte as the NumPy encoder does."""
    prec = abi.PRECISION_FAST
    terms = shade_terms(renderer, cfg, w, h, pose, prec)
    w0, _, w2 = _tile_widths(terms)
    narrow = (w0 <= 16) & (w2 <= 16)
    assert 0 < narrow.sum() < narrow.size, "the frame must exercise both encoder paths"
    _, st = render_pair(renderer, cfg, w, h, pose, prec)
    s = st.cpu().numpy()
    s = s[:tiles_ref.stream_bytes(s)]
    f = frame(cfg, w, h, pose, prec, abi.FORMAT_TILES)
    e = tiles_ref.encode(terms, tiles_ref.shade_header(f.light, f.material, False))
    n = narrow.size
    table_end, head = tiles_ref.HEADER_BYTES + 4 * n, tiles_ref.head_offset(n)
    assert s.size == e.size
    assert np.array_equal(s[:table_end], e[:table_end])
    assert np.array_equal(s[head:], e[head:])


def test_wide_tiles_decode_on_gpu(renderer):
    """Random 32-bit channel values: tiles whose base bits fill more than 64
    words (b0 + b1 + b2 up to 96), the words past the decoder's first vector
    load, read by each lane's own loads (ABI 10's pixel-by-pixel base bits);
    the stream sits at the very end of its buffer, so no load may run past
    the tiles' words."""
    import torch
    rng = np.random.default_rng(11)
    w, h = 24, 16
    a = np.ones((h, w, 4), dtype=np.float32)
    a[..., :3] = rng.integers(0, 2 ** 32, (h, w, 3), dtype=np.uint32).view(np.float32)
    s = tiles_ref.encode(a)
    n = tiles_ref.tiles_shape(w, h)[0] * tiles_ref.tiles_shape(w, h)[1]
    heads = np.frombuffer(s[tiles_ref.head_offset(n):tiles_ref.data_offset(n)].tobytes(),
                          dtype=np.uint32).reshape(n, 4)[:, 0]
    assert ((heads & 63) + (heads >> 6 & 63) + (heads >> 12 & 63) > 64).any()
    buf = torch.from_numpy(s.copy()).to(renderer.device)   # exactly the stream's bytes
    out = renderer.tiles_decode(buf, 1, buf.numel(), w, h)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), a)


# ---- malformed streams: the decoder must refuse, not fault --

def _stream_fields(st, n):
    """(table offsets, head word 0s, data offset, used) of a stream on the host."""
    s = st.cpu().numpy()
    used = int(s[:4].view(np.uint32)[0])
    table = s[tiles_ref.HEADER_BYTES:tiles_ref.HEADER_BYTES + 4 * n].view(np.uint32).copy()
    heads = s[tiles_ref.head_offset(n):tiles_ref.data_offset(n)].view(np.uint32).reshape(n, 4)
    return table, heads[:, 0].copy(), tiles_ref.data_offset(n), used


def _tile_mask(w, h, tiles):
    """Pixels (h, w) of the given tile indices (row-major 8x8 tiles, row 0 bottom)."""
    tx = (w + 7) // 8
    m = np.zeros((h, w), dtype=bool)
    for t in tiles:
        y, x = divmod(int(t), tx)
        m[8 * y:8 * y + 8, 8 * x:8 * x + 8] = True
    return m


def test_malformed_streams_are_refused(renderer):
    """A truncated or mismatched receive, a corrupted offset table, an
    impossible tile head and an escape field past its tile: the decode reads
    nothing outside the part, reports the part (SDF_TILES_BAD_* in its status
    word; SDF_E_COMM from the synchronous call), writes nothing for the bad
    tiles and decodes every other tile bit for bit."""
    import torch
    w, h = 160, 96
    ref, st = render_pair(renderer, "C3", w, h, 1, abi.PRECISION_EXACT)
    refn = ref.cpu().numpy()
    n = ((w + 7) // 8) * ((h + 7) // 8)
    table, heads, data0, used = _stream_fields(st, n)
    whole = [R.tiling(0, 1, h)]
    status = torch.zeros(1, dtype=torch.int32, device=renderer.device)

    def decode(buf, used_=None):
        out = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device=renderer.device)
        renderer.tiles_decode_checked(buf, 1, buf.numel(), w, h, whole, used=used_, out=out,
                                      status=status)
        torch.cuda.synchronize()
        return out.cpu().numpy(), int(status.cpu().numpy()[0]) & 0xFFFFFFFF

    # intact, with and without the agreed length: decodes, status 0
    out, code = decode(st, [used])
    assert code == 0 and same_bits(out, refn)
    # the receive got a different length than the header's: whole part skipped
    for bad_len in (used - 8, used + 8, 0):
        out, code = decode(st, [bad_len])
        assert code == abi.TILES_BAD_HEADER and np.isnan(out).all()
    with pytest.raises(RuntimeError, match="-5|COMM|collective"):
        renderer.tiles_decode_checked(st, 1, st.numel(), w, h, whole, used=[used - 8])
    # header claims more data than the part can hold
    b = st.clone()
    b[0:4] = torch.tensor([0xFF, 0xFF, 0xFF, 0x7F], dtype=torch.uint8)
    out, code = decode(b)
    assert code == abi.TILES_BAD_HEADER and np.isnan(out).all()
    # truncated: the stream's second half never arrived (zeros), its header
    # says so -- the tiles whose words lie past it are skipped
    half = (used // 2) & ~7
    b = st.clone()
    b[data0 + half:] = 0
    b[0:4] = torch.from_numpy(np.array([half], dtype=np.uint32).view(np.uint8)).to(b.device)
    nq = (heads >> 18) & 255
    cut = np.nonzero(table.astype(np.int64) + 8 * nq > half)[0]
    assert 0 < cut.size < n
    out, code = decode(b)
    m = _tile_mask(w, h, cut)
    assert code == abi.TILES_BAD_TILE
    assert np.isnan(out[m]).all() and same_bits(out[~m], refn[~m])
    # corrupted table entries and an impossible base width
    b = st.clone()
    bad = {3: 0xFFFFFF00, 17: used + 64, 40: 4}   # far away, past the data, misaligned
    t2 = table.copy()
    for t, v in bad.items():
        t2[t] = v
    b[tiles_ref.HEADER_BYTES:tiles_ref.HEADER_BYTES + 4 * n] = torch.from_numpy(
        t2.view(np.uint8)).to(b.device)
    h2 = heads.copy()
    h2[55] = (h2[55] & ~np.uint32(63)) | np.uint32(40)   # channel 0 base width 40 > 32
    hb = st[tiles_ref.head_offset(n):data0].cpu().numpy().view(np.uint32).reshape(n, 4).copy()
    hb[:, 0] = h2
    b[tiles_ref.head_offset(n):data0] = torch.from_numpy(hb.reshape(-1).view(np.uint8)).to(b.device)
    out, code = decode(b)
    m = _tile_mask(w, h, [*bad, 55])
    assert code == abi.TILES_BAD_TILE
    assert np.isnan(out[m]).all() and same_bits(out[~m], refn[~m])
    # an escape field pointing past its tile: a tile with escapes gets width
    # byte 255 (its fields' offsets then leave the tile's words)
    esc = np.nonzero((heads >> 26) & 7)[0]
    assert esc.size > 0
    t = int(esc[0])
    B = int((heads[t] & 63) + (heads[t] >> 6 & 63) + (heads[t] >> 12 & 63))
    P = int(bin(int(heads[t] >> 26) & 7).count("1"))
    at = data0 + int(table[t]) + 8 * (B + P)   # first byte of the bitstream: channel widths
    b = st.clone()
    b[at:at + P] = 255
    out, code = decode(b)
    assert code & abi.TILES_BAD_FIELD
    m = _tile_mask(w, h, [t])
    assert same_bits(out[~m], refn[~m])


def test_malformed_part_among_good_ones(renderer):
    """Several parts in one decode: only the malformed part is reported and
    left out; the other parts' rows come out bit-exact."""
    import torch
    world, w, h = 3, 96, 80
    f = frame("C3", w, h, 2, abi.PRECISION_FAST, abi.FORMAT_RGBA32F)
    whole, _ = renderer.render(f)
    tilings = [R.tiling(r, world, 8) for r in range(world)]
    stride = max(R.tiles_bytes(w, R.owned_rows(h, t)) for t in tilings)
    parts = torch.zeros(world * stride, dtype=torch.uint8, device=renderer.device)
    ft = frame("C3", w, h, 2, abi.PRECISION_FAST, abi.FORMAT_TILES)
    for r in range(world):
        renderer.render(ft, tilings[r], out=parts[r * stride:(r + 1) * stride])
    torch.cuda.synchronize()
    used = [int(parts[r * stride:r * stride + 4].cpu().numpy().view(np.uint32)[0])
            for r in range(world)]
    status = torch.zeros(world, dtype=torch.int32, device=renderer.device)
    out = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device=renderer.device)
    renderer.tiles_decode_checked(parts, world, stride, w, h, tilings,
                                  used=[used[0], used[1] + 16, used[2]], out=out, status=status)
    torch.cuda.synchronize()
    assert status.cpu().numpy().tolist() == [0, abi.TILES_BAD_HEADER, 0]
    o, wn = out.cpu().numpy(), whole.cpu().numpy()
    rows1 = np.zeros(h, dtype=bool)
    for y in range(h):
        rows1[y] = (y // 8) % world == 1
    assert np.isnan(o[rows1]).all() and same_bits(o[~rows1], wn[~rows1])
