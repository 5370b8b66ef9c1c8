import sys; sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import numpy as np, torch, tiles_ref
from sdf3d_amd import Renderer, abi, scenes, renderer as R
rd = Renderer("cuda:0")
w, h = 37, 23
f = scenes.config("REF", w, h, precision=abi.PRECISION_EXACT, pose=0)
ref, _ = rd.render(f)
f.params.output_format = abi.FORMAT_TILES
st, _ = rd.render(f)
torch.cuda.synchronize()
s = st.cpu().numpy(); host = ref.cpu().numpy()
used, n = np.frombuffer(s[:8].tobytes(), dtype=np.uint32)
print("used", used, "ntiles", n)
rs = tiles_ref.encode(host)
rused, rn = np.frombuffer(rs[:8].tobytes(), dtype=np.uint32)
print("ref used", rused, rn)
table = np.frombuffer(s[8:8+4*n].tobytes(), dtype=np.uint32)
print("table", table)
base = tiles_ref.data_offset(n)
rtable = np.frombuffer(rs[8:8+4*n].tobytes(), dtype=np.uint32)
for t in range(n):
    g = s[base+table[t]: base+table[t]+16].view(np.uint32)
    r = rs[base+rtable[t]: base+rtable[t]+16].view(np.uint32)
    gw = [g[0] & 255, g[0] >> 8 & 255, g[0] >> 16 & 255]; rw = [r[0] & 255, r[0] >> 8 & 255, r[0] >> 16 & 255]
    ok = np.array_equal(g, r)
    np_ = sum(rw)
    gp = s[base+table[t]+16: base+table[t]+16+8*np_].view(np.uint64)
    rp = rs[base+rtable[t]+16: base+rtable[t]+16+8*np_].view(np.uint64)
    if not ok or not np.array_equal(gp, rp):
        print("tile", t, "gpu hdr", gw, g[1:], "ref", rw, r[1:])
        print("  gpu planes", [hex(x) for x in gp[:6]]); print("  ref planes", [hex(x) for x in rp[:6]])
        break
else:
    print("all records equal")
try:
    d = tiles_ref.decode(s[:tiles_ref.stream_bytes(s)], w, h)
    print("numpy decode equal:", np.array_equal(d.view(np.uint32), host.view(np.uint32)))
except Exception as e:
    print("numpy decode error", e)
out = rd.tiles_decode(st, 1, st.numel(), w, h)
torch.cuda.synchronize()
o = out.cpu().numpy()
bad = np.argwhere(o.view(np.uint32) != host.view(np.uint32))
print("gpu decode mismatches", len(bad), bad[:5])
