#!/usr/bin/env python3
"""bench.py -- throughput of the SDF sphere-tracing hot path on MI355X.

One step = one frame of BASELINE.json's workload (default C4: the 8-primitive
smooth-min CSG scene with soft shadows, 5-tap AO and tetrahedral normals at
3840x2160, 128 max steps) in EXACT precision -- the oracle's fp32 operation
sequence, every pixel within north_star's 1e-4 of the reference restatement
(bit-exact at 4K); the fast precision (FMA contraction, hardware sqrt/rcp,
a few branch-flip pixels beyond 1e-4) is reported beside it as `fast` --
rendered by the HIP kernel through the C-ABI
(sdf_render), looped by the native frame driver (sdf_driver_*, C++).  With N
ranks (one process per GPU, torchrun) each rank renders its interleaved 8-row
blocks of the frame (rank 0 fewer: multigpu.choose_shares); the peers ship
them as lossless TILES streams to rank 0 over RCCL, and rank 0 decodes them
straight into the frame (sdf_tiles_decode_tilings).  Frames are pipelined
over 4 buffer sets on alternating streams (3 at N = 1): frame i ships while
frames i+1, i+2 render; HIP gets 8 hardware queues so that those streams do
not share one (GPU_MAX_HW_QUEUES, below).  Total work per step is one frame
whatever N is ("scaling": "strong").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C4]
                    [--precision fast|exact] [--no-cpu-baseline]

Prints ONE JSON line (rank 0).  `value` = frame pixels x K / max-over-ranks
wall time of the K timed steps, in Mpixels/s.  `roofline` is the render
kernel's executed FP32 rate (the hardware flop count of the committed PMC
summary, profiles/pmc_<cfg>_<prec>.json) over the kernel's average duration
measured with HIP events on the launch stream, against the 157.3 TFLOP/s FP32
vector peak, with the counter-based VALU busy of the same PMC run and, as
`alg_equiv`, the SURVEY.md 8(d) algorithmic count (oracle step counts in
tests/golden/stats_<cfg>_p0.npz) over the same time (see roofline()).
`cpu_baseline` times the CPU oracle (a restatement of the reference shader:
the reference's own OpenCL kernel is empty and no CPU OpenCL device exists)
on whole frames of the same workload, rank 0 at N=1 only; its last frame is
then the checker of the frames just timed (`parity.same_run`, `frame_verified`
at N=1: the last timed frame against it, pixel by pixel, after the timed
region).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent

# Hardware queues per process for HIP streams (read at HIP initialisation,
# before torch touches the GPU).  The frame driver keeps 3-4 render streams
# plus 2 communication streams; with HIP's default of 4 hardware queues some
# of them share a queue, whose FIFO order serialises their kernels: on one
# MI355X a rank-sized TILES share on 4 alternating streams took 0.073 ms per
# frame with 4 queues and 0.057 with 8 (tools/root_probe.py --streams,
# profiles/r02_hw_queues_C4.json).  A value set by the caller wins.  Not
# for the gloo rehearsals, whose ranks all share one GPU (up to 8 processes:
# HIP's default keeps their queue count at what one GPU was tested with).
def _gloo_rehearsal(argv):
    return any(a == "--backend=gloo" or (a == "--backend" and argv[i + 1:i + 2] == ["gloo"])
               for i, a in enumerate(argv))


# At N > 1 up to 8 render streams plus 2 communication streams (the
# Mandelbulb's 8 buffer sets, below): 12 queues (the pool allows up to 32).
if not _gloo_rehearsal(sys.argv[1:]):
    os.environ.setdefault("GPU_MAX_HW_QUEUES",
                          "12" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else "8")
sys.path.insert(0, str(ROOT))

METRIC = "Mpixels/s (primary+shadow+AO) at 3840×2160, 1/2/4/8 MI355X"
FP32_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: FP32 vector peak, 64 FLOP/clk/SIMD
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C4")
    # exact: the oracle's fp32 operation sequence, every pixel of the 4K
    # frame within north_star's 1e-4 (bit-exact); fast is reported beside it
    ap.add_argument("--precision", default="exact", choices=["fast", "exact"])
    ap.add_argument("--pose", type=int, default=0)
    ap.add_argument("--format", default="rgba32f", choices=["rgba32f", "rgba16f", "rgba8"],
                    help="framebuffer format of the assembled frame")
    ap.add_argument("--wire", default="auto", choices=["auto", "rgba", "rgb32f", "tiles"],
                    help="N>1: what ranks send; auto = tiles (lossless compressed RGB32F, "
                         "decoded into the frame on rank 0) for rgba32f frames, else the "
                         "frame format; rgb32f = uncompressed RGB, alpha restored")
    ap.add_argument("--shares", default="auto",
                    help="N>1 with the tiles wire: 'a:b' = rank 0 renders a 8-row blocks "
                         "and every other rank b per period of a + b (N - 1) (rank 0 "
                         "also decodes the others' streams); auto = the cost model of "
                         "multigpu.choose_shares; other wires always 1:1")
    ap.add_argument("--streams", type=int, default=0,
                    help="render streams / buffer sets of the frame driver (frame i on "
                         "stream i %% streams: a frame starts while the previous one's "
                         "slowest tiles finish); 1 serialises launches (profiling); "
                         "0 = 3 at N=1; at N>1 4, 8 for the Mandelbulb")
    ap.add_argument("--lag", type=int, default=2,
                    help="N>1: frames between a batch's last render and its gather (the "
                         "host reads the batch's agreed stream lengths that much later)")
    ap.add_argument("--batch", type=int, default=0,
                    help="N>1, native driver: frames per ship -- one RCCL length all-gather "
                         "and one send/recv group per `batch` frames (0 = 2; needs "
                         "streams %% batch == 0 and lag <= streams - batch)")
    ap.add_argument("--driver", default="native", choices=["native", "python"],
                    help="frame loop: native = sdf_driver_* (C++, RCCL called directly); "
                         "python = multigpu.FrameDriver over torch.distributed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exact", "--no-other", action="store_true",
                    help="N=1: skip the sub-object of the other precision (`fast` beside "
                         "the default exact headline, `exact` beside --precision fast)")
    ap.add_argument("--clock-warm-s", type=float, default=0.3,
                    help="seconds of render launches before anything is measured (the "
                         "GPU's clocks ramp up over ~0.1 s of load)")
    ap.add_argument("--cpu-sample-stride", type=int, default=1,
                    help="CPU baseline renders every k-th 8-row block of the frame")
    ap.add_argument("--cpu-frames", type=int, default=5)
    ap.add_argument("--no-verify", action="store_true",
                    help="N>1: skip the post-run check that rank 0's assembled frame equals "
                         "a single-device render bit for bit")
    ap.add_argument("--no-display", action="store_true",
                    help="skip the extra RGBA8-framebuffer measurement reported beside value")
    ap.add_argument("--comm-lib", default=None,
                    help="library with the RCCL symbols the native driver loads (default: the "
                         "librccl this process has mapped); with --backend gloo, a stand-in "
                         "such as tests/shmcomm/libshmcomm.so runs the native driver with "
                         "several ranks on one GPU")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to "
                         "rehearse several ranks on one GPU)")
    return ap.parse_args()


def rank_flops(frame, tiling, pose):
    """Algorithmic flops of one render launch over the rows `tiling` owns."""
    from sdf3d_amd import costmodel
    path = ROOT / "tests" / "golden" / f"stats_{frame.name}_p{pose}.npz"
    if not path.exists() or frame.scene.kind != 0:
        return None
    z = np.load(path)
    if int(z["width"]) != frame.params.width or int(z["height"]) != frame.params.height:
        return None
    H, B, run = frame.params.height, tiling.block_rows, max(tiling.block_run, 1)
    ys = [y for y in range(H) if (y // B) >= tiling.first_block
          and ((y // B) - tiling.first_block) % tiling.block_stride < run]
    c = costmodel.coefficients(frame)
    return c.flops(len(ys) * frame.params.width, z["row_sp"][ys].sum(), z["row_ss"][ys].sum())


def pmc_summary(cfg, precision):
    """The committed rocprofv3 PMC summary of the render kernel
    (profiles/pmc_<cfg>_<precision>.json, written by tools/pmc_traffic.py), or
    {} -- or {"stale": reason} when it was taken from another build of the
    kernel than the loaded library's (sdf_kernel_id)."""
    from sdf3d_amd import abi
    p = ROOT / "profiles" / f"pmc_{cfg}_{precision}.json"
    try:
        pmc = json.loads(p.read_text())
    except Exception:
        return {}
    prec = abi.PRECISION_FAST if precision == "fast" else abi.PRECISION_EXACT
    kid = abi.load_library().sdf_kernel_id(prec)
    kid = kid.decode() if kid else None
    if pmc.get("kernel_id") != kid:
        return {"stale": f"{p.name} was taken from kernel build {pmc.get('kernel_id')}, "
                         f"the library's is {kid}"}
    return pmc


def valu_cycles_per_unit():
    """gfx950 normalisation of SQ_ACTIVE_INST_VALU (tools/valu_busy_calib.py,
    profiles/r02_valu_busy_calib.json): SIMD cycles per counter unit, from
    kernels of pure full-rate VALU chains at full occupancy."""
    try:
        return float(json.loads((ROOT / "profiles" / "r02_valu_busy_calib.json")
                                .read_text())["cycles_per_unit"])
    except Exception:
        return None


def roofline(pmc, alg_flops, kavg_ms, store_bytes):
    """The render kernel against the FP32 VALU roofline.

    achieved = EXECUTED FP32 flops per launch -- the hardware count
    64 * (ADD + MUL + TRANS + 2 FMA) wave-instructions weighted by the VALU
    lane utilisation (SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU): the
    lanes EXEC left on) from the committed rocprofv3 PMC summary of the same
    kernel build (profiles/pmc_<cfg>_<prec>.json, tools/pmc_traffic.py,
    matched by sdf_kernel_id; a summary of another build gives frac null
    with the reason) -- over the live kernel time; frac <= 1 by
    construction.  valu_busy is the counter-based issue utilisation of the
    same PMC run (SQ_ACTIVE_INST_VALU x the calibrated gfx950 cycles per
    unit / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)); the counter counts a
    half-rate min/max/cmp as one unit, so it is a lower bound (a v_min-only
    chain reads 0.60).  alg_equiv is the SURVEY.md 8(d) counting rule (every
    primitive at every step, oracle step counts): exact culling skips
    evaluations that rule counts, so its `survey_rule_ratio` can exceed 1."""
    roof = {"bound": "valu", "achieved": None, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": None, "traffic": pmc.get("hbm_bytes_per_launch"),
            "kernel_ms": round(kavg_ms, 4),
            "store_GBps": round(store_bytes / (kavg_ms * 1e-3) / 1e9, 1),
            "kernel_id": pmc.get("kernel_id")}
    if "stale" in pmc:
        roof["frac_null_reason"] = pmc["stale"]
    ex = pmc.get("executed_flops_per_launch")
    if ex:
        ach = ex / (kavg_ms * 1e-3) / 1e12
        roof.update(achieved=round(ach, 2), frac=round(ach / FP32_PEAK_TFLOPS, 4),
                    executed_flops_per_launch=ex, valu_lane_util=pmc.get("valu_lane_util"),
                    basis="executed FP32 flops of the active lanes (PMC) / live kernel time")
    c = pmc.get("counters", {})
    cpu = valu_cycles_per_unit()
    if cpu and c.get("SQ_ACTIVE_INST_VALU") and c.get("GRBM_GUI_ACTIVE"):
        roof["valu_busy"] = round(cpu * c["SQ_ACTIVE_INST_VALU"]
                                  / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 4)
    if alg_flops is not None:
        alg = alg_flops / (kavg_ms * 1e-3) / 1e12
        # not a roofline fraction: the rule counts evaluations the exact
        # culling never performs, so this ratio may exceed 1
        roof["alg_equiv"] = {"flops_per_launch": alg_flops, "TFLOPs": round(alg, 2),
                             "survey_rule_ratio": round(alg / FP32_PEAK_TFLOPS, 4),
                             "note": "SURVEY 8(d) rule (every primitive at every step, oracle "
                                     "step counts) over the live kernel time, / 157.3 TF; exact "
                                     "culling skips evaluations it counts, so it may exceed 1 "
                                     "and is no roofline fraction"}
    if roof["achieved"] is None and alg_flops is None:
        return None
    return roof


def parity_summary(cfg, precision):
    """What the timed kernel satisfies: the committed full-size parity result
    of this configuration and precision (profiles/parity_fullsize.json,
    written by tests/test_gpu_parity.py test_full_size_pixel_parity on the
    GPU: the frame against a live oracle render, per pixel, outliers
    diagnosed by the forced-step replay), applied only to a library whose
    sdf_kernel_id matches the one it was taken from."""
    from sdf3d_amd import abi
    p = ROOT / "profiles" / "parity_fullsize.json"
    try:
        rec = json.loads(p.read_text()).get(f"{cfg}/{precision}")
    except Exception:
        rec = None
    if rec is None:
        return {"source": None, "note": f"no full-size parity result for {cfg}/{precision}"}
    prec = abi.PRECISION_FAST if precision == "fast" else abi.PRECISION_EXACT
    kid = abi.load_library().sdf_kernel_id(prec)
    kid = kid.decode() if kid else None
    out = {"precision": precision, "policy": rec.get("policy"), "pixels": rec.get("pixels"),
           "bit_exact": rec.get("bit_exact"), "outliers_over_1e-4": rec.get("outliers"),
           "replay_diagnosed": rec.get("replay_diagnosed"),
           "undiagnosed": rec.get("undiagnosed"), "over_0.05": rec.get("over_max_err"),
           "max_err": rec.get("max_err"), "undiagnosed_max_err": rec.get("undiagnosed_max_err"),
           "strict_policy_met": rec.get("policy") == "strict",
           "within_1e-4_everywhere": rec.get("outliers") == 0,
           "kernel_id": rec.get("kernel_id"), "source": f"profiles/{p.name}"}
    if rec.get("kernel_id") != kid:
        out["stale"] = (f"taken from kernel build {rec.get('kernel_id')}, the library's is {kid}")
    return out


def lib_bpp(frame):
    from sdf3d_amd import abi
    return abi.load_library().sdf_format_bytes(frame.params.output_format)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(frame, stride, frames):
    """The CPU oracle (the reference shader restated: its own OpenCL kernel
    is empty and no CPU OpenCL device exists) on whole frames (stride 1) or
    every stride-th 8-row block, OpenMP over the host threads this process
    may use, median of `frames` after one warm-up.
    Returns (the JSON object, the last oracle frame [rows, W, 4], the frame
    rows it holds): the frame is the checker of same_run_parity()."""
    import oracle
    from sdf3d_amd import renderer as R
    t = R.tiling(0, stride, 8) if stride > 1 else None
    n = oracle.default_threads()
    rows = oracle.owned_rows(frame.params.height, t)
    oracle.render(frame, t, nthreads=n, variant="baseline")          # warm-up
    times = []
    for _ in range(frames):
        t0 = time.perf_counter()
        rgba, _ = oracle.render(frame, t, nthreads=n, variant="baseline")
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    px = rows * frame.params.width
    H = frame.params.height
    ys = (np.arange(H) if stride <= 1 else
          np.array([y for y in range(H) if (y // 8) % stride == 0]))
    assert len(ys) == rows
    what = ("whole frames" if stride <= 1 else
            f"every {stride}th 8-row block ({rows} rows, {px} px)")
    return {"value": round(px / med / 1e6, 4), "unit": "Mpixels/s", "cores": n, "kind": "port",
            "cpu": cpu_model(), "nproc": os.cpu_count(),
            "sample": f"{frame.name} {frame.params.width}x{frame.params.height}, {what}, "
                      f"median of {frames} after 1 warm-up, {n} OpenMP threads (the process's "
                      f"CPU affinity), CPU oracle (oracle/oracle_core.h, gcc -O3 "
                      f"-march=x86-64-v4 -ffp-contract=off, no fast-math)",
            "seconds_per_sample": round(med, 3)}, rgba, ys


def same_run_parity(gpu_frame, ref, ys, precision):
    """The last TIMED frame (rank 0's, read back after the run) against the
    CPU oracle frame cpu_baseline() rendered of the same workload, on the
    rows the oracle rendered: per pixel, its largest per-channel |GPU -
    oracle|; an outlier exceeds north_star's 1e-4 (tests/parity.py's
    policy, without the replay diagnosis)."""
    g = gpu_frame.cpu().numpy()[ys]
    bits = (g.view(np.uint32) == ref.view(np.uint32)).all(axis=-1)
    err = np.abs(g.astype(np.float64) - ref.astype(np.float64)).max(axis=-1)
    err = np.where(bits, 0.0, err)                      # equal bits, NaN included
    nan = ~bits & np.isnan(err)
    err = np.where(nan, np.inf, err)
    out = int((err > 1e-4).sum())
    return {"precision": precision, "pixels": int(bits.size), "bit_exact": int(bits.sum()),
            "outliers_over_1e-4": out, "over_0.05": int((err > 0.05).sum()),
            "max_err": float(err.max()) if err.size else 0.0,
            "within_1e-4_everywhere": out == 0,
            "rows": ("all" if len(ys) == gpu_frame.shape[0] else
                     f"{len(ys)} rows (every block the CPU sample rendered)"),
            "what": "last timed frame of this run vs the CPU oracle frame rendered for "
                    "cpu_baseline (same scene, camera, size), compared after the timed region"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            sys.exit(f"--gpus {args.gpus} needs torchrun --nproc-per-node {args.gpus}")
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist
    from sdf3d_amd import Renderer, abi, scenes
    from sdf3d_amd import renderer as R
    from sdf3d_amd.multigpu import FrameDriver

    ndev = torch.cuda.device_count()
    dev_index = local_rank % ndev if args.backend == "gloo" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    prec = abi.PRECISION_FAST if args.precision == "fast" else abi.PRECISION_EXACT
    frame = scenes.config(args.config, precision=prec, pose=args.pose)
    frame.params.output_format = abi.FORMAT_NAMES[args.format]
    wire = args.wire
    if wire == "auto":
        wire = "tiles" if (world > 1 and args.format == "rgba32f") else "rgba"
    if wire in ("rgb32f", "tiles"):
        if args.format != "rgba32f":
            sys.exit(f"--wire {wire} needs --format rgba32f")
        # ranks render RGB (or its TILES stream), root assembles RGBA32F
        frame.params.output_format = abi.FORMAT_RGB32F if wire == "rgb32f" else abi.FORMAT_TILES
    W, H = frame.params.width, frame.params.height
    rd = Renderer(dev)
    # row shares: unequal only with the tiles wire (rank 0 decodes the rest)
    shares = (1, 1)
    if wire == "tiles" and world > 1:
        from sdf3d_amd.multigpu import choose_shares
        shares = (choose_shares(world) if args.shares == "auto"
                  else tuple(int(v) for v in args.shares.split(":")))
    t = R.tiling(rank, world, 8, shares=shares)
    t_equal = R.tiling(rank, world, 8)
    rows = R.owned_rows(H, t)
    # N > 1: a peer's share of the Mandelbulb (1/7 of the rows, 8-row blocks
    # interleaved) runs short kernels with long tails, and more frames in
    # flight fill them: its TILES share 0.154 / 0.123 / 0.113 / 0.110 ms on
    # 3 / 4 / 6 / 8 streams, where C4's is best at 4 (0.0668 against 0.0683
    # on 8; profiles/r06_peer_streams.jsonl)
    bulb = frame.scene.kind == abi.SCENE_MANDELBULB
    nbuf = args.streams or (3 if world == 1 else (8 if bulb else 4))
    batch = (args.batch or 2) if world > 1 else 1
    if nbuf % batch:
        batch = 1
    lag = min(args.lag, nbuf - batch) if nbuf > batch else 1

    open_drivers = []   # closed before the process group goes

    def native_driver(fr):
        """The C++ frame driver for frames of `fr`'s format, or None when it
        cannot serve them (then every rank falls back to the Python driver)."""
        from sdf3d_amd.driver import NativeFrameDriver
        f32 = fr.copy()
        if world > 1 or fr.params.output_format == abi.FORMAT_TILES:
            f32.params.output_format = abi.FORMAT_RGBA32F
        # N > 1: the TILES wire (lossless, decoded into an RGBA32F frame)
        wire_ok = world == 1 or fr.params.output_format == abi.FORMAT_TILES
        ok, drv = wire_ok and nbuf >= 2, None
        if ok:
            try:
                drv = NativeFrameDriver(f32, rank, world, dev, shares=shares, nbuf=nbuf,
                                        lag=lag if world > 1 else 1,
                                        dist=dist if world > 1 else None,
                                        rccl_path=args.comm_lib, batch=batch)
            except Exception as e:  # noqa: BLE001 - reported, then the fallback
                log(f"[bench] rank {rank}: native driver unavailable ({e})")
                ok = False
        if world > 1:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 0 and drv is not None:
                drv.close()
                drv, ok = None, False
        if drv is not None:
            open_drivers.append(drv)
        return drv

    fk = frame.copy()
    fk.params.output_format = abi.FORMAT_RGBA32F
    kbuf = rd.alloc(fk, t)[0]
    ks = torch.cuda.current_stream(dev)

    def warm_clocks():
        """Render launches for args.clock_warm_s seconds: the GPU takes longer
        than a few frames to leave its idle clocks (measured: 50 frames 0.406
        ms each, 200 frames 0.375), so every measurement below starts from
        its sustained clock -- after allocations, which idle it again."""
        tw = time.perf_counter()
        while True:
            for _ in range(10):
                rd.render(fk, t, out=kbuf, stream=ks)
            torch.cuda.synchronize(dev)
            if time.perf_counter() - tw >= args.clock_warm_s:
                break

    def timed_run(fr, steps, warmup):
        """warmup + `steps` timed frames of `fr` through a frame driver; returns
        (max-over-ranks seconds, per-launch kernel ms list, driver)."""
        # (gloo rehearsals share one GPU between ranks, which RCCL refuses)
        use_native = args.driver == "native" and nbuf >= 2 and (
            world == 1 or args.backend == "nccl" or args.comm_lib is not None)
        drv = native_driver(fr) if use_native else None
        if drv is not None:
            warm_clocks()
            for _ in range(warmup):
                drv.step()
            drv.drain()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                drv.step()
            drv.drain()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            if world > 1:
                e = torch.tensor([el], dtype=torch.float64, device=dev)
                dist.all_reduce(e, op=dist.ReduceOp.MAX)
                el = float(e.item())
            return el, [], drv
        tiles = fr.params.output_format == abi.FORMAT_TILES
        tr = t if tiles else t_equal

        def render_fn(out, stream):
            rd.render(fr, tr, out=out, stream=stream)

        if tiles:
            tilings = [R.tiling(r, world, 8, shares=shares) for r in range(world)]

            def tiles_fn(parts, nparts, pitch, w, h, b, out, stream, shares=None):
                rd.tiles_decode(parts, nparts, pitch, w, h, b, out=out, stream=stream,
                                tilings=tilings)

            # rank 0's own rows need no wire: rendered straight into the frame
            froot = fr.copy()
            froot.params.output_format = abi.FORMAT_RGBA32F
            troot = R.tiling(rank, world, 8, frame_rows=True, shares=shares)

            def root_fn(out, stream):
                rd.render(froot, troot, out=out, stream=stream)

            drv = FrameDriver(W, H, rank, world, dev, render_fn, tiles_fn,
                              dist=dist if world > 1 else None, wire="tiles",
                              nbuf=nbuf, root_render_fn=root_fn, shares=shares,
                              lag=lag)
        else:
            def deint_fn(parts, nparts, stride, w, h, b, out, stream):
                rd.deinterleave(parts, nparts, stride, w, h, b, out=out, stream=stream)

            drv = FrameDriver(W, H, rank, world, dev, render_fn, deint_fn,
                              dist=dist if world > 1 else None, nbuf=nbuf,
                              dtype=R.torch_dtype(fr.params.output_format),
                              wire_channels=R.channels(fr.params.output_format))
        k = steps + warmup
        e0 = [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        warm_clocks()
        for i in range(warmup):
            drv.step(i, e0[i], e1[i])
        drv.drain()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(warmup, k):
            drv.step(i, e0[i], e1[i])
        drv.drain()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            e = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el, [e0[i].elapsed_time(e1[i]) for i in range(warmup, k)], drv

    # the render kernel's own launch duration, for the roofline: the rank's
    # rows as RGBA32F, launches serialised on one stream with events around
    # each (in the pipelined frame loop a launch's events would also span
    # time queued behind the other streams' kernels)
    def kernel_avg_ms(fr):
        kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        warm_clocks()
        for a, b in kev:
            a.record(ks)
            rd.render(fr, t, out=kbuf, stream=ks)
            b.record(ks)
        torch.cuda.synchronize(dev)
        return sum(a.elapsed_time(b) for a, b in kev) / len(kev)

    kavg_ms = kernel_avg_ms(fk)
    log(f"[bench] rank {rank}/{world} {args.config} {W}x{H} rows={rows} "
        f"precision={args.precision} warmup={args.warmup} steps={args.steps}")
    elapsed, kernel_ms, drv = timed_run(frame, args.steps, args.warmup)
    k_steps = args.steps + args.warmup

    # the same workload written as the reference window's RGBA8 framebuffer:
    # 4 B/pixel on the gather wire instead of 12 (reported beside `value`)
    display = None
    if args.format == "rgba32f" and not args.no_display:
        fr8 = frame.copy()
        fr8.params.output_format = abi.FORMAT_RGBA8
        el8, km8, _ = timed_run(fr8, args.steps, args.warmup)
        display = {"format": "rgba8", "value": round(W * H * args.steps / el8 / 1e6, 3),
                   "fps": round(args.steps / el8, 2),
                   "ms_per_step": round(el8 / args.steps * 1e3, 4),
                   "render_ms_pipelined": round(sum(km8) / len(km8), 4) if km8 else None}

    # the same workload in the OTHER precision, through the same frame
    # driver, with its own kernel time, roofline and parity: `value` is the
    # exact precision by default (IEEE div/sqrt, no contraction: the oracle's
    # fp32 operation sequence, bit-exact with it on every pixel of the 4K
    # frame, tests/test_gpu_parity.py test_full_size_pixel_parity); the fast
    # precision (FMA contraction, hardware sqrt/rcp: within 1e-4 except at a
    # few branch flips, profiles/parity_fullsize.json) is this sub-object
    other, drv_other = None, None
    other_name = "fast" if prec == abi.PRECISION_EXACT else "exact"
    if world == 1 and not args.no_exact:
        fe = frame.copy()
        fe.params.precision = (abi.PRECISION_FAST if prec == abi.PRECISION_EXACT
                               else abi.PRECISION_EXACT)
        el_e, _, drv_other = timed_run(fe, args.steps, args.warmup)
        fek = fe.copy()
        fek.params.output_format = abi.FORMAT_RGBA32F
        kavg_e = kernel_avg_ms(fek)
        pmc_e = pmc_summary(args.config, other_name) if args.format == "rgba32f" else {}
        other = {"precision": other_name, "value": round(W * H * args.steps / el_e / 1e6, 3),
                 "unit": "Mpixels/s", "fps": round(args.steps / el_e, 2),
                 "ms_per_step": round(el_e / args.steps * 1e3, 4),
                 "kernel_ms": round(kavg_e, 4),
                 "roofline": roofline(pmc_e, rank_flops(fe, t, args.pose), kavg_e,
                                      rows * W * lib_bpp(frame)),
                 "parity": parity_summary(args.config, other_name)}

    # the same frames without the gather (scaling with and
    # without it): each rank renders its blocks only, max over ranks
    no_gather = None
    if world > 1:
        # the rank's own rows as RGBA32F, frames on alternating streams as in
        # the driver, nothing shipped
        fp = frame.copy()
        fp.params.output_format = abi.FORMAT_RGBA32F
        bufs = [rd.alloc(fp, t)[0] for _ in range(3)]
        strs = [torch.cuda.Stream(device=dev) for _ in range(3)]
        for i in range(args.warmup):
            rd.render(fp, t, out=bufs[i % 3], stream=strs[i % 3])
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            rd.render(fp, t, out=bufs[i % 3], stream=strs[i % 3])
        torch.cuda.synchronize(dev)
        dist.barrier()
        e = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el_ng = float(e.item())
        no_gather = {"value": round(W * H * args.steps / el_ng / 1e6, 3),
                     "fps": round(args.steps / el_ng, 2),
                     "ms_per_step": round(el_ng / args.steps * 1e3, 4)}
        del bufs

    verified = None
    if world > 1 and not args.no_verify and rank == 0:
        # outside the timed region: the assembled frame of the last step must
        # equal a whole-frame render on this device (pixels are independent)
        whole = scenes.config(args.config, precision=prec, pose=args.pose)
        whole.params.output_format = abi.FORMAT_NAMES[args.format]
        ref, _ = rd.render(whole)
        got = (drv.read_frame(k_steps - 1) if hasattr(drv, "read_frame")
               else drv.frame(k_steps - 1))
        torch.cuda.synchronize(dev)
        verified = bool(torch.equal(got.view(torch.uint8), ref.view(torch.uint8)))
        log(f"[bench] assembled frame == single-device frame: {verified}")

    flops = rank_flops(frame, t, args.pose)

    native = hasattr(drv, "read_frame")
    driver_desc = ("native (sdf_driver_*, C++)" if native
                   else "python (multigpu.FrameDriver, torch.distributed)")
    if native:
        gather_desc = (f"per batch of {batch} frames: one RCCL all-gather of the TILES stream "
                       "lengths + one RCCL send/recv group of exactly those bytes to rank 0; "
                       "sdf_tiles_decode_tilings per frame")
    else:
        gather_desc = (f"{'RCCL' if args.backend == 'nccl' else 'gloo'} gather to rank 0 + "
                       + ("sdf_tiles_decode_tilings" if wire == "tiles" else "sdf_deinterleave"))
    if rank == 0:
        value = W * H * args.steps / elapsed / 1e6
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mpixels/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.config}: {frame.meta['description']}",
                       "width": W, "height": H, "max_steps": frame.params.max_steps,
                       "precision": args.precision, "pose": args.pose,
                       "format": args.format, "wire": wire if world > 1 else None,
                       "tiling": (f"8-row blocks, rank 0 {shares[0]} / others {shares[1]} per "
                                  f"period of {shares[0] + shares[1] * (world - 1)}"
                                  if world > 1 else "whole frame"),
                       "gather": gather_desc if world > 1 else None,
                       "driver": driver_desc,
                       "streams": nbuf, "lag": lag if world > 1 else None,
                       "batch": batch if (world > 1 and native) else None},
            "fps": round(args.steps / elapsed, 2),
            "frame_verified": verified,
            "display_rgba8": display,
            other_name: other,
            "no_gather": no_gather,
            "kernel_ms": round(kavg_ms, 4),
            # host (CPU) time of the frame loop's own calls per frame, waits
            # for the GPU / peers excluded (native driver only)
            "driver_host_us_per_frame": drv.stats()["host_us_per_frame"] if native else None,
            # the same split by the driver's enqueue calls (renders with the
            # TILES compaction, length all-gathers, send/recv groups, decodes)
            "driver_enqueue_us_per_frame": (drv.stats()["enqueue_us_per_frame"] if native
                                            else None),
        }
        pmc = (pmc_summary(args.config, args.precision)
               if world == 1 and args.format == "rgba32f" else {})
        out["roofline"] = roofline(pmc, flops, kavg_ms, rows * W * lib_bpp(frame))
        # the full-size parity of the precision `value` was timed in
        out["parity"] = parity_summary(args.config, args.precision)
        if world == 1 and not args.no_cpu_baseline:
            log("[bench] cpu baseline ...")
            out["cpu_baseline"], ref, ys = cpu_baseline(frame, args.cpu_sample_stride,
                                                        args.cpu_frames)
            # parity as a fact of this run: the frames just timed against the
            # oracle frame the baseline rendered (no extra timed work)
            if native and args.format == "rgba32f":
                got = drv.read_frame(k_steps - 1)
                torch.cuda.synchronize(dev)
                sr = same_run_parity(got, ref, ys, args.precision)
                out["parity"]["same_run"] = sr
                out["frame_verified"] = sr["within_1e-4_everywhere"]
                out["frame_verified_what"] = ("N=1: the last timed frame within 1e-4 of the CPU "
                                              "oracle on every compared pixel (parity.same_run)")
                if other is not None and hasattr(drv_other, "read_frame"):
                    got = drv_other.read_frame(k_steps - 1)
                    torch.cuda.synchronize(dev)
                    other["parity"]["same_run"] = same_run_parity(got, ref, ys, other_name)
                log(f"[bench] same-run parity: {sr['bit_exact']}/{sr['pixels']} bit-exact, "
                    f"{sr['outliers_over_1e-4']} over 1e-4, max err {sr['max_err']:.3g}")
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    for d in open_drivers:
        d.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
