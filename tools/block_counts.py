#!/usr/bin/env python3
"""Dynamic instruction attribution of a render kernel -- measurement tooling,
not product.

The production translation unit (e.g. render_exact.hip, its own build.py
flags plus -gline-tables-only, which leaves the instruction stream unchanged:
checked by `build`) is compiled to gfx950 assembly.  In the chosen kernel
every basic block (a label, or the fall-through after a branch) gets a
counter: the first active lane of the wave adds 1 to the block's wave count
in LDS, and every active lane adds 1 to its lane count.  The sequence uses
only VGPRs above the kernel's own allocation (v64..v71; the kernel keeps its
59-64) and no SGPR, VCC, SCC or M0, so the kernel's own instructions -- all
of them, in the same order -- are exactly the production kernel's.  At every
s_endpgm the wave adds its LDS counters into a global array placed after the
frame in the output buffer.  Multiplying the per-block counts by each block's
static instruction classes gives the kernel's dynamic mix (checked against
the PMC counters of the production build), and the instructions' inline
stacks (llvm-symbolizer on the un-instrumented code object) assign it to
source constructs.

    python tools/block_counts.py build [--unit render_exact.hip] [--kernel SUBSTR]
    python tools/block_counts.py run --config C4 --precision exact   (GPU)
    python tools/block_counts.py report gpurun_out/blocks_C4_exact.json
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shlex
import subprocess
import sys
from collections import Counter, defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "tools" / "_variants" / "blocks"
LLVM = Path("/opt/rocm/lib/llvm/bin")
KERNEL_C4 = "FixedSceneIJLi56ELi1ELi17ELi33ELi41ELi49ELi25ELi1EEEELb0ELb0E"
SPARE = 64          # first spare VGPR: v64..v71
NEXT_FREE = 72


# ---- build ------------------------------------------------------------------

def pipeline(unit: str, flags: list[str], workdir: Path) -> list[list[str]]:
    from sdf3d_amd import build as B
    cmd = [B._hipcc(), *B.COMMON, *flags, "-gline-tables-only", "-I", str(B.OBJ), "-c",
           str(B.CSRC / unit), "-o", "unit.o", "-###", "-save-temps"]
    r = subprocess.run(cmd, cwd=workdir, capture_output=True, text=True, check=True)
    return [shlex.split(l) for l in r.stderr.splitlines() if l.startswith(' "')]


def classify(op: str) -> str:
    op = re.sub(r"_(e32|e64|dpp|sdwa)$", "", op)
    if not op.startswith("v_"):
        return "salu" if op.startswith("s_") else "other_mem"
    if op.endswith("_f64") or "_f64_" in op:
        return "f64"
    if op in ("v_rsq_f32", "v_rcp_f32", "v_sqrt_f32", "v_log_f32", "v_exp_f32", "v_rcp_iflag_f32",
              "v_sin_f32", "v_cos_f32"):
        return "trans"
    if re.match(r"v_(fma|fmac|fmaak|fmamk|mad|mac)_f32", op) or op.startswith("v_pk_fma_f32"):
        return "fma"
    if re.match(r"v_(add|sub|subrev)_f32", op):
        return "add"
    if re.match(r"v_mul_f32", op):
        return "mul"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "cmp"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if re.match(r"v_(min|max|min3|max3|med3)_f32", op):
        return "minmax"
    if op.startswith(("v_mov", "v_readlane", "v_readfirstlane", "v_writelane")):
        return "mov"
    return "valu_other"


def instrument(lines: list[str], kernel: str, frame_off: int, rgba_karg: int):
    """Insert the block counters into `kernel` of the assembly `lines`;
    returns (new lines, blocks: list of {id, label, ins: [(op, text, idx)]})."""
    # spare VGPRs above the kernel's own (its .num_vgpr), 8 of them
    global SPARE, NEXT_FREE
    # ".set K.num_vgpr, N", or "max(N, .Lcallee.num_vgpr, ...)" when the kernel
    # makes calls (the library log/pow fall-backs): the largest of them
    sets = {m.group(1): m.group(2) for l in lines
            for m in [re.match(r"\s*\.set (\S+)\.num_vgpr, (.+)$", l)] if m}

    def num_vgpr(sym, depth=0):
        rhs = sets[sym]
        vals = [int(x) for x in re.findall(r"(?<![\w.])(\d+)(?![\w.])", rhs)]
        vals += [num_vgpr(c, depth + 1) for c in re.findall(r"(\.?[\w.]+?)\.num_vgpr", rhs)
                 if depth < 4 and c in sets]
        return max(vals)
    nv = num_vgpr(kernel)
    SPARE = (nv + 3) // 4 * 4
    NEXT_FREE = SPARE + 8
    start = next(i for i, l in enumerate(lines) if re.match(rf"^{re.escape(kernel)}:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start + 1:end]
    for l in body:
        m = re.search(r"lgkmcnt\((\d+)\)", l)
        if m and int(m.group(1)) != 0:
            raise SystemExit(f"kernel waits on lgkmcnt({m.group(1)}): counters would disturb it")
        for m in re.finditer(r"\bv(\d+)\b|v\[(\d+):(\d+)\]", l):
            hi = int(m.group(1) or m.group(3))
            if hi >= SPARE:
                raise SystemExit(f"kernel uses v{hi}, above its .num_vgpr {nv}")
    blocks, out = [], []
    state = {"open": False}

    def open_block(label):
        b = len(blocks)
        blocks.append({"id": b, "label": label, "ins": []})
        v = SPARE
        out.extend([
            f"\tv_mbcnt_lo_u32_b32 v{v+2}, exec_lo, 0",
            f"\tv_mbcnt_hi_u32_b32 v{v+2}, exec_hi, v{v+2}",
            f"\tv_sub_u32 v{v+2}, 1, v{v+2}",
            f"\tv_max_i32 v{v+2}, 0, v{v+2}",
            f"\tv_mov_b32 v{v+3}, {4 * b}",
            f"\tds_add_u32 v{v+3}, v{v+2}",
            f"\tv_mov_b32 v{v+4}, 1",
            f"\tds_add_u32 v{v+3}, v{v+4} offset:LANEOFF",
        ])
        state["open"] = True

    def flush():
        v = SPARE
        seq = ["\ts_mov_b64 exec, -1",
               f"\tv_readfirstlane_b32 s0, v{v}",
               f"\tv_readfirstlane_b32 s1, v{v+1}",
               f"\ts_load_dwordx2 s[0:1], s[0:1], {rgba_karg:#x}",
               "\ts_waitcnt vmcnt(0) lgkmcnt(0)",
               f"\ts_add_u32 s0, s0, {frame_off & 0xffffffff:#x}",
               f"\ts_addc_u32 s1, s1, {frame_off >> 32:#x}",
               f"\tv_mbcnt_lo_u32_b32 v{v+2}, -1, 0",
               f"\tv_mbcnt_hi_u32_b32 v{v+2}, -1, v{v+2}",
               f"\tv_lshlrev_b32 v{v+2}, 2, v{v+2}"]
        for c in range(NCHUNK[0]):
            seq += [f"\tds_read_b32 v{v+3}, v{v+2} offset:{256 * c}",
                    f"\tv_add_u32 v{v+4}, {256 * c:#x}, v{v+2}",
                    "\ts_waitcnt lgkmcnt(0)",
                    f"\tglobal_atomic_add v{v+4}, v{v+3}, s[0:1]"]
        seq += ["\ts_waitcnt vmcnt(0)"]
        return seq

    NCHUNK = [0]
    pending_entry = True
    for l in body:
        s = l.strip()
        is_ins = l.startswith("\t") and s and not s.startswith((".", ";"))
        if re.match(r"^\.LBB\d+_\d+:", l):
            out.append(l)
            open_block(l.split(":")[0])
            continue
        if pending_entry and is_ins:
            # kernel entry: keep the kernarg pointer, zero the counters
            v = SPARE
            out.extend([f"\tv_mov_b32 v{v}, s0", f"\tv_mov_b32 v{v+1}, s1",
                        f"\tv_mov_b32 v{v+5}, 0",
                        f"\tv_mbcnt_lo_u32_b32 v{v+2}, -1, 0",
                        f"\tv_mbcnt_hi_u32_b32 v{v+2}, -1, v{v+2}",
                        f"\tv_lshlrev_b32 v{v+2}, 2, v{v+2}", "ZEROLDS",
                        "\ts_waitcnt lgkmcnt(0)"])
            open_block("entry")
            pending_entry = False
        if is_ins:
            op = s.split()[0]
            if op == "s_endpgm":
                if not state["open"]:
                    open_block(f"after_{len(blocks)}")
                blocks[-1]["ins"].append(op)
                out.append("FLUSH")
                out.append(l)
                state["open"] = False
                continue
            if not state["open"]:
                open_block(f"after_{len(blocks)}")
            blocks[-1]["ins"].append(op)
            out.append(l)
            if op.startswith("s_cbranch") or op == "s_branch" or op.startswith("s_setpc"):
                state["open"] = False
            continue
        out.append(l)
    nb = len(blocks)
    NCHUNK[0] = (2 * nb + 63) // 64
    lds = 4 * 64 * NCHUNK[0]
    final = []
    for l in out:
        if l == "FLUSH":
            final.extend(flush())
        elif l == "ZEROLDS":
            final.extend(f"\tds_write_b32 v{SPARE+2}, v{SPARE+5} offset:{256 * c}"
                         for c in range(NCHUNK[0]))
        else:
            final.append(l.replace("offset:LANEOFF", f"offset:{4 * nb}"))
    new = lines[:start + 1] + final + lines[end:]
    # resources of this kernel: VGPRs, LDS
    text = "\n".join(new)
    kd = text.index(f".amdhsa_kernel {kernel}")
    kd_end = text.index(".end_amdhsa_kernel", kd)
    seg = text[kd:kd_end]
    seg = re.sub(r"\.amdhsa_group_segment_fixed_size \d+",
                 f".amdhsa_group_segment_fixed_size {lds}", seg)
    seg = re.sub(r"\.amdhsa_next_free_vgpr \S+", f".amdhsa_next_free_vgpr {NEXT_FREE}", seg)
    seg = re.sub(r"\.amdhsa_accum_offset \S+", f".amdhsa_accum_offset {NEXT_FREE}", seg)
    text = text[:kd] + seg + text[kd_end:]
    # metadata (YAML): this kernel's entry
    mi = text.index(f".name:           {kernel}") if f".name:           {kernel}" in text else \
        text.index(f".name: {kernel}")
    ms = text.rfind("\n  - .agpr_count", 0, mi)
    me = text.find("\n  - .agpr_count", mi)
    me = me if me > 0 else text.index("amdhsa.target", mi)
    meta = text[ms:me]
    meta = re.sub(r"\.group_segment_fixed_size: \d+", f".group_segment_fixed_size: {lds}", meta)
    meta = re.sub(r"\.vgpr_count:\s+\d+", f".vgpr_count:     {NEXT_FREE}", meta)
    text = text[:ms] + meta + text[me:]
    # the symbolic resource counts newer assemblers emit (.set <k>.num_vgpr)
    text = re.sub(rf"(\.set {re.escape(kernel)}\.num_vgpr), \d+", rf"\1, {NEXT_FREE}", text)
    return text.split("\n"), blocks, lds


def rgba_kernarg_offset() -> int:
    src = OUT / "off.cpp"
    src.write_text('#include <cstdio>\n#include <cstddef>\n#include "kernel_args.h"\n'
                   'int main(){printf("%zu", offsetof(sdf::RenderArgs, a) + '
                   'offsetof(sdf::KernelArgs, rgba));}\n')
    exe = OUT / "off"
    from sdf3d_amd import build as B
    subprocess.run([B._hipcc(), "-std=c++17", "-I", str(ROOT / "sdf3d_amd" / "csrc"), str(src),
                    "-o", str(exe)], check=True, capture_output=True)
    return int(subprocess.run([str(exe)], capture_output=True, text=True).stdout)


def symbolize(kname: str) -> list:
    """Inline stacks (leaf first: [function, file:line]) of every instruction
    of `kname` in the un-instrumented code object, in address order."""
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", f"--disassemble-symbols={kname}",
                          str(OUT / "orig.hsaco")], capture_output=True, text=True,
                         check=True).stdout
    addrs = []
    for l in dis.splitlines():
        m = re.match(r"^\s+(\S+)\s.*//\s*([0-9A-Fa-f]+):", l)
        if m:
            addrs.append(int(m.group(2), 16))
    sym = subprocess.run([str(LLVM / "llvm-symbolizer"), "--inlining",
                          f"--obj={OUT / 'orig.hsaco'}"], input="\n".join(hex(x) for x in addrs),
                         capture_output=True, text=True).stdout.strip().split("\n\n")
    stacks = []
    for entry in sym:
        frames = entry.strip().split("\n")
        st = []
        for j in range(0, len(frames) - 1, 2):
            fn = re.sub(r"^(void|float|bool|int|V3|float4) ", "", frames[j].strip())
            loc = frames[j + 1].strip()
            m = re.match(r".*/([^/]+):(\d+):(\d+)", loc)
            st.append([fn[:90], f"{m.group(1)}:{m.group(2)}" if m else loc])
        stacks.append(st)
    return stacks


def cmd_symbolize(a):
    meta = json.loads((OUT / "blocks_meta.json").read_text())
    meta["stacks"] = symbolize(meta["kernel"])
    assert len(meta["stacks"]) == sum(len(b["ins"]) for b in meta["blocks"])
    (OUT / "blocks_meta.json").write_text(json.dumps(meta))
    print(f"re-symbolized {len(meta['stacks'])} instructions")


def cmd_build(a):
    from sdf3d_amd import build as B
    OUT.mkdir(parents=True, exist_ok=True)
    work = Path(os.environ.get("TMPDIR", "/tmp")) / "sdf_blocks_work"   # not in the tree
    work.mkdir(exist_ok=True)
    flags = dict(B.UNITS)[a.unit]
    cmds = pipeline(a.unit, flags, work)
    dev_s = next(c[c.index("-o") + 1] for c in cmds if "-S" in c and "amdgcn-amd-amdhsa" in c)
    i_s = next(i for i, c in enumerate(cmds) if "-S" in c and "amdgcn-amd-amdhsa" in c)
    for c in cmds[:i_s + 1]:
        subprocess.run(c, cwd=work, check=True)
    orig = (work / dev_s).read_text().split("\n")
    # the production stream (no -g) must be the same instructions
    prod = work / "prod.s"
    subprocess.run([B._hipcc(), *B.COMMON, *flags, "-I", str(B.OBJ), "--offload-device-only",
                    "-S", str(B.CSRC / a.unit), "-o", str(prod)], check=True, capture_output=True)
    kname = next(re.match(r"^(\S+):", l).group(1) for l in orig
                 if re.match(rf"^_Z\S*render\S*{re.escape(a.kernel)}\S*:", l))

    def stream(lines):
        s = next(i for i, l in enumerate(lines) if l.startswith(kname + ":"))
        e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
        return [l.split(";")[0].strip() for l in lines[s:e]
                if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    so, sp = stream(orig), stream(prod.read_text().split("\n"))
    same = so == sp
    # the same instructions up to register numbering (the register allocator
    # may number differently with line tables): the block structure, every
    # opcode and every non-register operand equal -- the counts are exact
    reg = re.compile(r"\b[vsa]\[\d+:\d+\]|\b[vsa]\d+\b")
    same_ops = len(so) == len(sp) and all(reg.sub("R", x) == reg.sub("R", y) for x, y in zip(so, sp))
    print(f"kernel {kname}: -gline-tables-only stream identical to production: {same}"
          f" (up to register numbering: {same_ops})")
    if not same_ops:
        raise SystemExit("debug line tables changed the code: attribution would not be exact")
    # the un-instrumented code object (symbolization)
    asm_i = next(i for i, c in enumerate(cmds) if "-cc1as" in c and "amdgcn-amd-amdhsa" in c)
    lld_i = next(i for i, c in enumerate(cmds) if "lld" in c[0])
    dev_o = cmds[asm_i][cmds[asm_i].index("-o") + 1]
    dev_out = cmds[lld_i][cmds[lld_i].index("-o") + 1]
    subprocess.run(cmds[asm_i], cwd=work, check=True)
    subprocess.run(cmds[lld_i], cwd=work, check=True)
    os.replace(work / dev_out, OUT / "orig.hsaco")
    # instrument, then the rest of the pipeline
    frame_off = a.frame_bytes
    new, blocks, lds = instrument(orig, kname, frame_off, rgba_kernarg_offset())
    (work / dev_s).write_text("\n".join(new))
    for c in cmds[i_s + 1:]:
        subprocess.run(c, cwd=work, check=True)
    objs = []
    for src, _ in B.UNITS:
        o = B.OBJ / (Path(src).stem + ".o")
        objs.append(str(work / "unit.o") if src == a.unit else str(o))
    lib = OUT / "libsdf3d.so"
    subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib),
                    *objs, "-lhiprtc", "-ldl"], check=True)
    stacks = symbolize(kname)
    ninst = sum(len(b["ins"]) for b in blocks)
    print(f"{len(blocks)} blocks, {ninst} instructions; symbolized {len(stacks)}; LDS {lds} B")
    meta = {"unit": a.unit, "kernel": kname, "frame_bytes": frame_off, "lds": lds,
            "nblocks": len(blocks), "blocks": blocks,
            "stacks": stacks if len(stacks) == ninst else None,
            "note": "stacks[i] = inline frames (leaf first) of the i-th kernel instruction "
                    "in block order"}
    (OUT / "blocks_meta.json").write_text(json.dumps(meta))
    if len(stacks) != ninst:
        print(f"warning: {len(stacks)} symbolized vs {ninst} instructions")
    print(f"wrote {lib} and {OUT / 'blocks_meta.json'}")


# ---- run (GPU) ----------------------------------------------------------------

def cmd_run(a):
    import ctypes as C

    import torch
    from sdf3d_amd import abi, scenes
    meta = json.loads((OUT / "blocks_meta.json").read_text())
    lib = abi.load_library(OUT / "libsdf3d.so")
    prec = abi.PRECISION_EXACT if a.precision == "exact" else abi.PRECISION_FAST
    f = scenes.config(a.config, precision=prec, pose=a.pose)
    W, H = f.params.width, f.params.height
    frame = W * H * 16
    assert frame == meta["frame_bytes"], (frame, meta["frame_bytes"])
    nb = meta["nblocks"]
    ncnt = meta["lds"] // 4
    buf = torch.zeros(frame // 4 + ncnt, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(a.launches):
        rc = lib.sdf_render(C.byref(f.scene), C.byref(f.camera), C.byref(f.light),
                            C.byref(f.material), C.byref(f.params), None,
                            C.c_void_p(buf.data_ptr()), None, C.c_void_p(s.cuda_stream))
        abi.check(rc, "sdf_render")
    torch.cuda.synchronize()
    cnt = buf[frame // 4:].cpu().numpy().astype("int64") // a.launches
    waves = ((W + 7) // 8) * ((H + 7) // 8)
    res = {"config": a.config, "precision": a.precision, "pose": a.pose, "waves": waves,
           "kernel": meta["kernel"], "wave_counts": cnt[:nb].tolist(),
           "lane_counts": cnt[nb:2 * nb].tolist()}
    out = Path(a.out or f"gpurun_out/blocks_{a.config}_{a.precision}.json")
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res))
    print(f"wrote {out}: entry block waves {cnt[0]} (expected {waves})")


# ---- report ---------------------------------------------------------------------

# shade_pixel's stages: render_kernel.inc line ranges found from anchors in
# its source (so the table follows edits of the file)
ANCHORS = [("// quad = ((2x+1)/W - 1,", "setup: quad, ray"), ("// raymarch, :86-103", "primary march"),
           ("// normal, :134-155", "normal"), ("// ambient occlusion (extension)", "AO"),
           ("// Blinn-Phong, :200-204", "Blinn-Phong"), ("// soft shadow, :105-132", "shadow setup"),
           ("tlim = scene.shadow_limit(", "shadow lit-tail setup"), ("if (!lit)", "shadow march"),
           ("const float dif = gclamp(ndl", "colour terms")]


def _stages():
    lines = (ROOT / "sdf3d_amd" / "csrc" / "render_kernel.inc").read_text().split("\n")
    start = next(i for i, l in enumerate(lines) if "__device__ __forceinline__ float4 shade_pixel(" in l)
    marks = []
    for key, name in ANCHORS:
        i = next(j for j in range(start, len(lines)) if key in lines[j])
        marks.append((i + 1, name))
    end = next(j for j in range(start, len(lines)) if lines[j].startswith("}")) + 1
    return [(a, (marks[k + 1][0] - 1) if k + 1 < len(marks) else end, name)
            for k, (a, name) in enumerate(marks)]


STAGES = None


def stage(stack) -> str:
    global STAGES
    if STAGES is None:
        STAGES = _stages()
    for fn, loc in stack:
        if fn.startswith("shade_pixel") and loc.startswith("render_kernel.inc:"):
            ln = int(loc.split(":")[1])
            for a, b, name in STAGES:
                if a <= ln <= b:
                    return name
            return f"shade_pixel:{ln}"
    for fn, _ in stack:
        if fn.startswith(("render_body", "store_pixel", "pixel_value", "shade_colour")):
            return "store / index"
    return "entry / scene setup"


KEYS = [("log_fast", "cr_log"), ("log_round_ok", "cr_log"), ("cr_log", "cr_log"),
        ("bulb_roots", "bulb: map"), ("bulb_map", "bulb: map"), ("bulb_step", "bulb: map"),
        ("bulb_de", "bulb: DE"), ("de_div", "bulb: DE"), ("mandelbulb", "bulb: orbit loop"),
        ("div3_prepared", "bulb: (p - c) / scale"), ("BulbScene::local", "bulb: (p - c) / scale"),
        ("BulbScene::eval", "bulb: eval"),
        ("sqrt_fast", "cr_sqrt"), ("sqrt_guard", "cr_sqrt"), ("cr_sqrt", "cr_sqrt"),
        ("rcp_fast", "rcp_fast"), ("div_refined", "Markstein division"),
        ("div3", "Markstein division"), ("div_scaled", "smin: h = n / k"),
        ("div_prepared", "smin: h = n / k"), ("smin", "smin"), ("spec_pow", "spec pow"),
        ("fdiv", "IEEE division"), ("cr_log", "cr_log"), ("cull_dist2", "culling: fresh test"),
        ("wave_near", "culling: fresh test"), ("box_core", "primitive SDF"),
        ("sd_", "primitive SDF"), ("prim_ct", "primitive SDF"),
        ("step_cached", "culling: per-primitive"), ("taps_step", "culling: per-primitive (taps)"),
        ("suffix_cached", "culling: per-primitive"), ("::march", "culling: cluster"),
        ("march", "culling: cluster"), ("taps_suffix", "culling: per-primitive (taps)"),
        ("max_of", "taps: max of accumulators"), ("::taps", "culling: cluster (taps)"),
        ("taps", "culling: cluster (taps)"), ("head", "scene head (plane)"),
        ("plane_clear", "lit tail"), ("shadow_limit", "lit tail"), ("normalize", "normalize"),
        ("shade_colour", "shade colour"), ("store_pixel", "store"),
        ("TetraTaps", "tap points"), ("AOTaps", "tap points")]


def constructs(stack) -> list[str]:
    """Labels of the frames of an instruction's inline stack (leaf first)
    that name a source construct."""
    out = []
    for fn, loc in stack:
        for key, label in KEYS:
            if key in fn:
                if not out or out[-1] != label:
                    out.append(label)
                break
    return out


def construct(stack) -> str:
    c = constructs(stack)
    if c:
        return c[0] if len(c) == 1 else f"{c[0]} < {c[1]}"
    for fn, loc in stack:
        if fn.startswith("shade_pixel"):
            return f"shade_pixel {loc}"
    return f"{stack[-1][0][:30] if stack else '?'} {stack[0][1] if stack else ''}"


def cmd_report(a):
    meta = json.loads((OUT / "blocks_meta.json").read_text())
    res = json.loads(Path(a.result).read_text())
    waves = res["waves"]
    wc, lc = res["wave_counts"], res["lane_counts"]
    stacks = meta["stacks"]
    by_class = Counter()
    by_construct = defaultdict(Counter)
    by_stage = defaultdict(Counter)
    by_stage_con = defaultdict(Counter)
    by_line = Counter()
    lanes = Counter()
    k = 0
    for b in meta["blocks"]:
        n = wc[b["id"]]
        for op in b["ins"]:
            c = classify(op)
            by_class[c] += n
            st = stacks[k] if stacks else []
            con = construct(st)
            by_construct[con][c] += n
            by_stage[stage(st)][c] += n
            by_stage_con[(stage(st), con)][c] += n
            if c not in ("salu", "other_mem"):
                by_line[(st[0][1] if st else "?", op)] += n
                lanes[c] += lc[b["id"]]
            k += 1
    valu = ("trans", "fma", "add", "mul", "cmp", "cndmask", "minmax", "mov", "valu_other", "f64")
    tot = sum(by_class[c] for c in valu)
    print(f"{res['config']} {res['precision']}: VALU/wave {tot / waves:.1f}  "
          + "  ".join(f"{c} {by_class[c] / waves:.1f}" for c in valu)
          + f"  salu {by_class['salu'] / waves:.1f}")
    flop = sum(by_class[c] for c in ("fma", "add", "mul"))
    print(f"  full-rate flop {flop / waves:.1f}, trans {by_class['trans'] / waves:.1f}, "
          f"other {(tot - flop - by_class['trans']) / waves:.1f}")
    rows = []
    for con, cc in by_construct.items():
        v = sum(cc[c] for c in valu) / waves
        rows.append((v, con, {c: round(cc[c] / waves, 1) for c in valu if cc[c]}))
    rows.sort(reverse=True)
    for v, con, cc in rows[:a.top]:
        print(f"  {v:8.1f}  {con:45s} {cc}")
    def eq(cc):   # issue cost in plain-VALU units: a transcendental costs 2
        return sum(cc[c] for c in valu) + cc["trans"]
    print("by stage (VALU/wave, trans, other = cmp/cndmask/minmax/mov/int/f64):")
    stage_rows = []
    for st, cc in sorted(by_stage.items(), key=lambda kv: -sum(kv[1][c] for c in valu)):
        v = sum(cc[c] for c in valu) / waves
        oth = sum(cc[c] for c in ("cmp", "cndmask", "minmax", "mov", "valu_other", "f64")) / waves
        stage_rows.append({"stage": st, "valu_per_wave": round(v, 1),
                           "trans": round(cc["trans"] / waves, 1), "other": round(oth, 1),
                           "issue_units": round(eq(cc) / waves, 1)})
        print(f"  {v:8.1f}  trans {cc['trans'] / waves:6.1f} other {oth:6.1f}  {st}")
    sc_rows = []
    for (st, con), cc in sorted(by_stage_con.items(), key=lambda kv: -eq(kv[1])):
        v = sum(cc[c] for c in valu) / waves
        if v < 0.5:
            continue
        sc_rows.append({"stage": st, "construct": con, "valu_per_wave": round(v, 1),
                        "issue_units": round(eq(cc) / waves, 1),
                        "classes": {c: round(cc[c] / waves, 1) for c in valu if cc[c]}})
    print("by stage x construct (top):")
    for r in sc_rows[:a.top]:
        print(f"  {r['valu_per_wave']:8.1f} ({r['issue_units']:6.1f})  {r['stage']:22s} "
              f"{r['construct']:45s} {r['classes']}")
    print("top source lines (leaf) x opcode, VALU/wave:")
    for (line, op), n in by_line.most_common(a.top):
        print(f"  {n / waves:8.1f}  {line:28s} {op}")
    if a.json:
        out = {"config": res["config"], "precision": res["precision"], "pose": res["pose"],
               "kernel": res["kernel"], "waves": waves,
               "valu_per_wave": round(tot / waves, 1),
               "classes_per_wave": {c: round(by_class[c] / waves, 1) for c in (*valu, "salu")},
               "stages": stage_rows, "stage_constructs": sc_rows,
               "constructs": [{"construct": con, "valu_per_wave": round(v, 1), "classes": cc}
                              for v, con, cc in rows],
               "lines": [{"line": l, "op": op, "per_wave": round(n / waves, 2)}
                         for (l, op), n in by_line.most_common(200)]}
        Path(a.json).write_text(json.dumps(out, indent=1))
        print(f"wrote {a.json}")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("build")
    b.add_argument("--tag", default="blocks", help="variant directory under tools/_variants")
    b.add_argument("--unit", default="render_exact.hip")
    b.add_argument("--kernel", default=KERNEL_C4)
    b.add_argument("--frame-bytes", type=int, default=3840 * 2160 * 16)
    r = sub.add_parser("run")
    r.add_argument("--tag", default="blocks", help="variant directory under tools/_variants")
    r.add_argument("--config", default="C4")
    r.add_argument("--precision", default="exact")
    r.add_argument("--pose", type=int, default=0)
    r.add_argument("--launches", type=int, default=1)
    r.add_argument("--out", default=None)
    sy = sub.add_parser("symbolize")
    sy.add_argument("--tag", default="blocks")
    p = sub.add_parser("report")
    p.add_argument("--tag", default="blocks", help="variant directory under tools/_variants")
    p.add_argument("result")
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--json", default=None)
    a = ap.parse_args()
    global OUT
    OUT = ROOT / "tools" / "_variants" / a.tag
    {"build": cmd_build, "run": cmd_run, "report": cmd_report,
     "symbolize": cmd_symbolize}[a.cmd](a)


if __name__ == "__main__":
    main()
