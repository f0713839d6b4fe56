#!/usr/bin/env python3
"""Throughput of the MI355X StereoAnywhere forward on synthetic 540x960 pairs.

    python bench.py [--gpus N --steps K --warmup W] [--config cfg2|cfg4|cfg3|cfg5]
        (N > 1 without torchrun: bench.py starts the N ranks itself, one child process per GPU)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): stereo pairs/s at 540x960 "D=192" (a label: the reference volume
is all-pairs over W/4), configs[1]: batch 4 per GPU, padded to 544x960
(test.py:206-213), 22 GRU iterations, published flags, seeded weights, fp32.
A step = one test_mode forward over the rank's batch, inputs resident in HBM.
Weak scaling: every rank runs its own batch of 4; value = all pairs / max-over-ranks time.

Also reported (rank 0):
  roofline      the dominant hand-written kernel, timed live with HIP events on its
                launch stream inside the timed region (libsa_hip sa_timing_*),
                algorithmic bytes or flops per launch / mean launch time vs MI355X peak
  cpu_baseline  the oracle CPU restatement (torch CPU + numpy, parity-pinned to the
                reference) on one 544x960 pair, all host threads, N=1 only: one warm-up
                run, then the median of 3; cfg1 (256x512, 8 iters) the same
                way beside it; the CPU model string and the thread count are reported

  --config cfg4  configs[3]: batch 64 sharded 8-way = 8 pairs per GPU (seeds 1 + 8 * rank ..), the
                 same step otherwise; at world size 8 the global batch is configs[3]'s 64, below it
                 the line is configs[3]'s per-rank workload (the scaling curve needs an 8-GPU node)

Box state: the GPU's sysfs clock levels, power and temperatures before and after the timed
region, and sclk / power sampled every 100 ms during it (box_state; the run-to-run spread of
the headline is attributed against these).

Tiled configs (separate lines, not the headline):
  --config cfg3  Middlebury-H-sized synthetic pair 1000x1400 (padded 1024x1408), middlebury
                 preset (672x1120 tiles, overlap 112 -> 128): 3 tiles, 32 iterations
  --config cfg5  Booster full-res synthetic pair 3008x4112 (padded 3008x4128), booster preset
                 (1120x896 tiles, overlap 224) under CPUOffloadWrapper: 25 tiles, 32 iterations
  A step = one image through the tiler (TileWrapper with batch_tiles, the reference's own
  option: every tile has the preset's size, so the tiles run as one batch), stitched.
  epe_vs_reference  EPE of this build vs the reference's own disparity (golden vector,
                544x960, 22 iterations) on identical inputs and weights
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from stereoanywhere_amd import _native as N  # noqa: E402
from stereoanywhere_amd import dist as D  # noqa: E402
from stereoanywhere_amd import ops  # noqa: E402
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

PUBLISHED = dict(use_truncate_vol=True, use_aggregate_mono_vol=True, vol_n_masks=8, n_additional_hourglass=0,
                 vol_downsample=0, mirror_conf_th=0.98, mirror_attenuation=0.9, lrc_th=1.0, normal_gain=10)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8 TB/s spec
FP32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_*_f32 dense peak
# fp32 products as f16 hi/lo pairs on v_mfma_f32_16x16x16_f16: 4 f16 products per fp32 product at
# half the f16 MFMA peak (the 16x16x16 form issues at 16 cycles per SIMD, scripts/micro/mfma_rate.hip)
SPLIT_MFMA_PEAK_TFS = 2 * FP32_MFMA_PEAK_TFS


def step_costs(B: int, H4: int, W4: int, iters: int, C: int = 256):
    """Algorithmic work of one forward step per hand-written kernel family:
    {kernel: (unit, amount per step)} — minimal bytes each launch must move (HBM-bound
    kernels) or flops it must do (compute-bound ones).  Derivations in DESIGN.md §4."""
    px = B * H4 * W4                      # 1/4-res pixels
    vol = px * W4                         # cost-volume cells
    lv = [W4 >> i for i in range(4)]
    return {
        # fp32 MFMA: 2*C flops per volume cell (a1); epilogue work (trunc, pyramid) is free
        "corr_volume_pyramid": ("TFLOP/s", 2.0 * vol * C),
        # per pixel: 2 volumes x 4 levels x (2r+2) cells read, coords read, and (convc1 fused)
        # 2 x 64 channels of relu(convc1(taps)) written
        "corr_lookup": ("GB/s", iters * px * (2 * 4 * 10 * 4 + 4 + 2 * 64 * 4)),
        # the sheared copies of the two pyramids (large volumes only): every level cell read
        # from the row layout and written once
        "corr_shear": ("GB/s", 2 * 2 * px * sum(lv) * 4),
        "mono_masked_volume": ("GB/s", 8 * vol * 4 + px * 2 * 4 * 4),
        # two aggregated volumes read once, four maps written
        "softargmin_conf": ("GB/s", 2 * vol * 4 + 4 * px * 4),
        # three joint L/R maps read once
        "weighted_lsq": ("GB/s", 3 * 2 * px * 4),
        "convex_upsample": ("GB/s", px * (144 + 1) * 4 + px * 16 * 4),
        # the whole mono hourglass + classifier (11 fused conv launches; fp32 FMA), flops
        # per full-res volume cell: full res 1x1x1 24->8, 3x3x3 8->8 (x2), 8->2;
        # 1/8 (stride-2 outputs) 8->16, 16->16 (x3), 1x1x1 48->16;  1/64: 16->32, 32->32.
        # (the two vol_apply launches timed in this family move < 2% of its bytes)
        "conv3d_fused": ("TFLOP/s", 2.0 * vol * (24 * 8 + 2 * 27 * 8 * 8 + 27 * 8 * 2
                                                 + (27 * 8 * 16 + 3 * 27 * 16 * 16 + 48 * 16) / 8
                                                 + (27 * 16 * 32 + 27 * 32 * 32) / 64)),
    }


def pmc_traffic(kernel: str, batch: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic_*.json, made by scripts/pmc_traffic.py on this bench config)."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_b{batch}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f).get(kernel)
    return None if rec is None else rec["hbm_bytes_per_launch"]


F16_DENSE_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense (spec)


def _gpu_sysfs(device):
    """The sysfs directory of this process's GPU (by PCI address), or None."""
    import glob
    try:
        pr = torch.cuda.get_device_properties(device)
        addr = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}."
    except Exception:
        return None
    for d in sorted(glob.glob("/sys/bus/pci/devices/*")):
        if os.path.basename(d).startswith(addr) and os.path.exists(os.path.join(d, "pp_dpm_sclk")):
            return d
    return None


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _dpm_current(text):
    """The starred line of a pp_dpm_* table ('1: 2400Mhz *') -> MHz."""
    if not text:
        return None
    for line in text.splitlines():
        if line.rstrip().endswith("*"):
            try:
                return float(line.split(":", 1)[1].strip().rstrip("*").strip().lower().replace("mhz", ""))
            except ValueError:
                return None
    return None


def box_state(d):
    """One snapshot of the GPU's DPM levels, power and temperatures (sysfs; None where unreadable)."""
    import glob
    if d is None:
        return None
    out = {"sysfs": d, "sclk_mhz": _dpm_current(_read(os.path.join(d, "pp_dpm_sclk"))),
           "mclk_mhz": _dpm_current(_read(os.path.join(d, "pp_dpm_mclk"))),
           "fclk_mhz": _dpm_current(_read(os.path.join(d, "pp_dpm_fclk")))}
    for hw in sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*"))):
        for name in ("power1_average", "power1_input"):
            v = _read(os.path.join(hw, name))
            if v and v.lstrip("-").isdigit():
                out["power_w"] = int(v) / 1e6
                break
        cap = _read(os.path.join(hw, "power1_cap"))
        if cap and cap.isdigit():
            out["power_cap_w"] = int(cap) / 1e6
        for t in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
            lab = _read(t.replace("_input", "_label")) or os.path.basename(t)
            v = _read(t)
            if v and v.lstrip("-").isdigit():
                out[f"temp_{lab}_c"] = int(v) / 1e3
        for fq in sorted(glob.glob(os.path.join(hw, "freq*_input"))):
            lab = _read(fq.replace("_input", "_label")) or os.path.basename(fq)
            v = _read(fq)
            if v and v.isdigit():
                out[f"{lab}_hwmon_mhz"] = int(v) / 1e6
    return out


class BoxSampler:
    """sclk / power sampled from sysfs every ``period`` s on a thread while the timed steps run."""

    def __init__(self, d, period: float = 0.1):
        import threading
        self.d, self.period, self.samples = d, period, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True) if d else None

    def _run(self):
        while not self._stop.is_set():
            st = box_state(self.d)
            self.samples.append({k: st.get(k) for k in ("sclk_mhz", "power_w")})
            self._stop.wait(self.period)

    def __enter__(self):
        if self._t:
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t:
            self._t.join()

    def summary(self):
        res = {"samples": len(self.samples)}
        for k in ("sclk_mhz", "power_w"):
            v = [x[k] for x in self.samples if x.get(k) is not None]
            if v:
                res[k] = {"min": min(v), "mean": sum(v) / len(v), "max": max(v)}
        return res


def clock_probe(device):
    """The in-kernel shader clock under a dense MFMA load (sa_clock_probe: median over waves of
    delta s_memtime / delta s_memrealtime x 100 MHz; MI355X_MICROARCH.md 'DVFS give-back' 6), which
    sysfs's pp_dpm_sclk does not show; ~3 ms of work on every CU.  None if unavailable."""
    import ctypes
    try:
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        mhz, ms = ctypes.c_double(), ctypes.c_double()
        N.call("sa_clock_probe", 2 * cus, 40000, ctypes.byref(mhz), ctypes.byref(ms))
        return {"mfma_clock_mhz": mhz.value, "probe_ms": ms.value}
    except Exception as e:   # (an older library, or no GPU)
        return {"error": str(e)[:200]}


def make_inputs(B, H, W, Hp, Wp, D, seed0, device):
    pb = synth.synthetic_batch(B, H, W, D, seed0=seed0)
    out = {}
    for k in ("left", "right", "mono_left", "mono_right"):
        x, _ = synth.pad_to_multiple(pb[k], 32)
        assert x.shape[-2:] == (Hp, Wp)
        out[k] = torch.from_numpy(np.ascontiguousarray(x)).to(device)
    return out


def _cgroup_cpus():
    """CPUs the cgroup's CFS quota grants (cpu.max 'quota period'), or None without a quota."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        return None


def host_cpu_share() -> dict:
    """The host CPUs this process may use: the affinity mask, capped by the cgroup's CPU quota
    when there is one; OMP_NUM_THREADS (16 on the GPU box) is reported beside them and is
    the fallback cap when neither the mask nor a quota bounds the share (os.cpu_count() reports
    the whole machine there)."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    env = os.environ.get("OMP_NUM_THREADS")
    omp = int(env) if env and env.isdigit() and int(env) > 0 else None
    if quota is not None:
        use = min(aff, quota)
    elif omp is not None and aff >= (os.cpu_count() or aff):
        use = omp    # the mask is the whole machine: stay within the box's stated share
    else:
        use = aff
    return {"threads": use, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "omp_num_threads": omp}


def host_threads() -> int:
    return host_cpu_share()["threads"]


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _time_oracle(sd, H, W, iters, D, runs):
    """One warm-up forward, then ``runs`` timed ones; returns the sorted wall times."""
    from oracle import model_ref as M

    pair = synth.synthetic_batch(1, H, W, D, seed0=1)
    t = [torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")]
    M.forward(sd, *t, iters=iters)
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        M.forward(sd, *t, iters=iters)
        times.append(time.perf_counter() - t0)
    return sorted(times)


def cpu_baseline(iters: int, H: int, W: int, runs: int = 3, cfg1: bool = True):
    """The oracle restatement (parity-pinned to the reference) on the box's host threads:
    one warm-up, then the median of ``runs`` single-pair forwards, at the bench shape and
    (cfg1) at configs[0] (256x512, 8 iterations)."""
    from oracle import model_ref as M

    share = host_cpu_share()
    torch.set_num_threads(share["threads"])
    sd = M.load_state_dict_seeded(0)
    ts = _time_oracle(sd, H, W, iters, 192.0, runs)
    med = ts[len(ts) // 2]
    res = {"value": 1.0 / med, "unit": "pairs/s", "cores": torch.get_num_threads(), "kind": "port",
           "cpu_model": cpu_model(), "cpu_share": share,
           "sample": f"1 pair 1x{H}x{W}, {iters} iters, oracle (torch CPU convs + numpy hot path); "
                     f"1 warm-up + median of {runs}: {', '.join(f'{x:.2f}' for x in ts)} s"}
    if cfg1:
        t1 = _time_oracle(sd, 256, 512, 8, 64.0, runs)
        res["cfg1"] = {"value": 1.0 / t1[len(t1) // 2], "unit": "pairs/s",
                       "sample": f"1 pair 1x256x512, 8 iters; 1 warm-up + median of {runs}: "
                                 f"{', '.join(f'{x:.2f}' for x in t1)} s"}
    return res


def rank_report(per_rank_s, steps: int, gather_ms: float, gather_bytes: int, backend: str) -> dict:
    """N > 1: what makes the line explain itself (the only data-path collective is the
    metric all_gather after the timed region): each rank's timed-region length per step (the value
    divides by the slowest), which rank that was, and the all_gather's own latency and size.
    per_rank_s: each rank's own K steps, from the opening barrier to its own device sync (before the
    closing barrier, which equalises the bracketed times)."""
    ms = [t / steps * 1e3 for t in per_rank_s]
    slow = max(range(len(ms)), key=lambda i: ms[i])
    return {"per_rank_ms_per_step": ms, "slowest_rank": slow, "spread": max(ms) / min(ms),
            "gather_ms": gather_ms, "gather_bytes": gather_bytes, "backend": backend}


def cpu_baseline_tile(cfg, iters: int, runs: int = 3):
    """Tiled configs: the oracle on ONE tile of the config (bounded sample): one warm-up
    run, then the median of ``runs``."""
    share = host_cpu_share()
    torch.set_num_threads(share["threads"])
    sd = M_load()
    th, tw = cfg["tile_hw"]
    ts = _time_oracle(sd, th, tw, iters, cfg["D"], runs)
    dt = ts[len(ts) // 2]
    n = cfg["unique_tiles"]
    return {"value": 1.0 / dt, "unit": "tiles/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": cpu_model(), "cpu_share": share,
            "sample": f"1 tile 1x{th}x{tw}, {iters} iters, oracle; 1 warm-up + median of {runs}: "
                      f"{', '.join(f'{x:.1f}' for x in ts)} s (one image = {n} unique tile forwards -> "
                      f"{1.0 / (dt * n):.4f} images/s)"}


def M_load():
    from oracle import model_ref as M
    return M.load_state_dict_seeded(0)


def epe_vs_reference(model, device):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_util import load_fixture, regenerate_inputs  # golden data only

    fix = load_fixture("cfg2_544x960_it22.npz")
    pair = regenerate_inputs(fix, 1, 544, 960, 192.0)
    t = [torch.from_numpy(pair[k]).to(device) for k in ("left", "right", "mono_left", "mono_right")]
    flow_up, _ = model(*t, iters=22, test_mode=True)
    disp = -flow_up[:, 0].cpu().numpy()
    return float(np.abs(disp.astype(np.float64) - fix["disparity"]).mean())


def epe_vs_reference_tiled(model, device, config: str):
    """Against the reference at the tiled configs' own 32 iterations (tests/golden/tiled32.npz):
    cfg3 = config 3's whole padded 1024x1408 image through this build's tiler (6 tiles, 3 unique)
    vs the reference TileWrapper + model; cfg5 = one 896x1120 booster tile through the model."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_util import load_fixture  # golden data only
    from stereoanywhere_amd import tiler

    fix = load_fixture("tiled32.npz")
    step = int(fix["row_step"])
    if config == "cfg3":
        H, W, tw, th, ov, seed = (int(v) for v in fix["cfg3.geom"])
        pair = synth.synthetic_batch(1, H, W, float(fix["cfg3.D"]), seed0=seed)
        t = [torch.from_numpy(pair[k]).to(device) for k in ("left", "right", "mono_left", "mono_right")]
        got = tiler.TileWrapper(model, tile_width=tw, tile_height=th, overlap=ov, batch_tiles=True)(
            *t, iters=32, test_mode=True)
        ref = fix["cfg3.out"]
    else:
        H, W, seed = (int(v) for v in fix["booster_tile.geom"])
        pair = synth.synthetic_batch(1, H, W, float(fix["booster_tile.D"]), seed0=seed)
        t = [torch.from_numpy(pair[k]).to(device) for k in ("left", "right", "mono_left", "mono_right")]
        got = -model(*t, iters=32, test_mode=True)[0]
        ref = fix["booster_tile.out"]
    got = got[0, 0, ::step].cpu().numpy()
    return float(np.abs(got.astype(np.float64) - ref).mean())


# the tiled BASELINE configs: padded image, preset, iterations
TILED = {
    "cfg3": dict(index=2, image=(1000, 1400), preset="middlebury", iters=32, D=256.0, offload=False),
    "cfg5": dict(index=4, image=(3008, 4112), preset="booster", iters=32, D=512.0, offload=True),
}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(gpus: int):
    """``--gpus N`` (N > 1) outside torchrun: start N child ranks of this same command, one per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), poll them and return the first
    non-zero exit status (0 when every rank succeeded).  As torchrun does, the first rank that fails
    ends the others (SIGTERM, then SIGKILL after a grace period): the survivors would otherwise block
    for ever in a collective with the dead rank.  None: nothing to launch (N = 1, or already a rank of
    a torchrun / self-launched world).  The parent touches no GPU: the children are fresh
    interpreters started before any HIP call (no exec from a GPU process)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    port = _free_port()
    procs = []
    for rank in range(gpus):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(gpus),
                   LOCAL_WORLD_SIZE=str(gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    import time
    first_bad = None
    while True:
        rcs = [p.poll() for p in procs]
        bad = [c for c in rcs if c not in (None, 0)]
        if bad and first_bad is None:
            first_bad = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.monotonic() + 15.0
            while any(p.poll() is None for p in procs) and time.monotonic() < deadline:
                time.sleep(0.1)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            rcs = [p.wait() for p in procs]
        if all(c is not None for c in rcs):
            break
        time.sleep(0.1)
    if first_bad is not None or any(c != 0 for c in rcs):
        print(f"bench: rank exit codes {rcs}", file=sys.stderr)
        return first_bad if first_bad is not None else next(c for c in rcs if c != 0)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg4", "cfg3", "cfg5"],
                    help="cfg2 = the headline (configs[1]); cfg4 = configs[3]'s 8 pairs per GPU; "
                         "cfg3 / cfg5 = the tiled configs")
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU (configs[1]: 4, configs[3]: 8)")
    ap.add_argument("--iters", type=int, default=None, help="GRU iterations (default: the config's)")
    ap.add_argument("--height", type=int, default=540)
    ap.add_argument("--width", type=int, default=960)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-epe", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches instead of hipGraph replay")
    ap.add_argument("--one-stream", action="store_true",
                    help="every step eager on one stream, the whole batch per launch (the schedule of the "
                         "instrumented steps: rocprof per-launch times and PMC bytes comparable with the live ones)")
    ap.add_argument("--miopen-find", type=int, default=0,
                    help="let MIOpen time its conv algorithms per shape (torch cudnn.benchmark)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="graph instances in flight (PipelinedForward): consecutive batches overlap; 1: one "
                         "forward at a time")
    ap.add_argument("--conv3d-mfma", type=int, default=None, choices=[0, 1],
                    help="the hourglass's stride-1 8->8 / 16->16 convs on split-f16 MFMA (1) or on the F(4,3) "
                         "VALU kernel (0); default: ops.CONV3D_MFMA")
    ap.add_argument("--lookup-mfma", type=int, default=None, choices=[0, 1],
                    help="the fused lookups' convc1 on fp32 MFMA (1) or on the VALU (0); default: the library's "
                         "(sa_lookup_get_mfma)")
    ap.add_argument("--lookup-form", type=int, default=None, choices=[0, 1, 2, 3],
                    help="the sheared lookup's work split (sa_lookup_set_shear_dual): 0 one volume per "
                         "thread, 1 both, 2 spread over a 4-wave block, 3 over 8 waves (the library's default)")
    ap.add_argument("--w4-split", type=int, default=None, choices=[0, 1],
                    help="F(4x4) convs on the split kernel (1) or fp32 MFMA (0); default: ops.W4_SPLIT")
    ap.add_argument("--direct-split", type=int, default=None, choices=[0, 1],
                    help="direct convs on split products (1) or fp32 MFMA (0); default: ops.DIRECT_SPLIT")
    ap.add_argument("--direct-small", type=int, default=None, choices=[0, 1],
                    help="the context encoder's small stride-2 stages on the direct kernel (1) or MIOpen (0); "
                         "default: encoders.DIRECT_SMALL")
    ap.add_argument("--conv1x1", type=int, default=None, choices=[0, 1],
                    help="the 1x1 convs on sa_conv1x1 (1) or F.conv2d / rocBLAS (0); default: ops.CONV1X1")
    ap.add_argument("--split-guard", type=int, default=None, choices=[0, 1],
                    help="the split kernel's f16 range guard (default ops.SPLIT_GUARD; 0 for A/B timing only)")
    ap.add_argument("--opts", default="",
                    help="ScheduleOptions overrides for A/B runs, e.g. fuse_flow_head=0,loop_parts=1")
    ap.add_argument("--offload-release", type=int, default=0, choices=[0, 1],
                    help="cfg5: CPUOffloadWrapper empties the allocator cache after each call (1, the "
                         "reference's behaviour) or keeps its pools (0, HBM-resident; the other setting is "
                         "timed beside it)")
    ap.add_argument("--wino4-min-blocks", type=int, default=None,
                    help="F(4x4) for launches of at least this many blocks (default: ops._WINO4_MIN_BLOCKS)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rendezvous only: every rank joins the process group and rank 0 prints the ranks that "
                         "reported (checks the multi-rank launch without a model or a GPU)")
    args = ap.parse_args()
    # --gpus N > 1 without a torchrun environment: this process becomes the launcher of N ranks
    # (before anything touches the GPU); under torchrun the world size must match --gpus
    rc = self_launch(args.gpus)
    if rc is not None:
        raise SystemExit(rc)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE {world_env}: the line would report "
                         f"{world_env} GPU(s); launch with --nproc-per-node {args.gpus} (or without torchrun)")
    if args.dry_run:
        r = D.init_from_env(os.environ.get("SA_DIST_BACKEND", "nccl"))
        if os.environ.get("SA_DIST_BACKEND", "nccl") == "nccl":
            torch.cuda.set_device(r.local_rank)
        dev = torch.device("cuda", r.local_rank) if os.environ.get("SA_DIST_BACKEND", "nccl") == "nccl" else None
        if os.environ.get("SA_DRYRUN_FAIL_RANK") == str(r.rank):   # (tests: a rank that dies after joining)
            raise SystemExit(3)
        # the timed-region bookkeeping of a real run on stand-in steps (rank r sleeps 5 (r + 1) ms per step)
        D.barrier(r)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            time.sleep(5e-3 * (r.rank + 1))
        own = time.perf_counter() - t0
        D.barrier(r)
        per_rank = D.gather_scalars(own, r, dev)
        tg = time.perf_counter()
        got = D.gather_metrics(torch.tensor([[float(r.rank), float(r.world)]], dtype=torch.float64, device=dev), r)
        gather_ms = (time.perf_counter() - tg) * 1e3
        D.barrier(r)
        if r.is_main:
            line = {"dry_run": True, "n_gpus": r.world, "ranks": [int(v) for v in got[:, 0].tolist()],
                    "worlds": sorted({int(v) for v in got[:, 1].tolist()})}
            if r.world > 1:
                line["rank_timing"] = rank_report(per_rank, args.steps, gather_ms, got.numel() * 8,
                                                  os.environ.get("SA_DIST_BACKEND", "nccl"))
            if not args.no_cpu_baseline:   # (a tiny oracle sample: the key's plumbing, not a baseline)
                line["cpu_baseline"] = cpu_baseline(1, 64, 128, runs=1, cfg1=False)
            print(json.dumps(line))
        return
    if args.split_guard is not None:
        ops.SPLIT_GUARD = bool(args.split_guard)
    if args.batch is None:
        args.batch = 8 if args.config == "cfg4" else 4
    if args.wino4_min_blocks is not None:
        ops._WINO4_MIN_BLOCKS = args.wino4_min_blocks
    if args.w4_split is not None:
        ops.W4_SPLIT = bool(args.w4_split)
    if args.conv3d_mfma is not None:
        ops.CONV3D_MFMA = bool(args.conv3d_mfma)
    if args.lookup_mfma is not None:
        from stereoanywhere_amd import _native as _N
        _N.lib().sa_lookup_set_mfma(int(args.lookup_mfma))
    if args.lookup_form is not None:
        from stereoanywhere_amd import _native as _N
        _N.lib().sa_lookup_set_shear_dual(int(args.lookup_form))
    if args.direct_split is not None:
        ops.DIRECT_SPLIT = bool(args.direct_split)
    if args.direct_small is not None:
        from stereoanywhere_amd import encoders as _E
        _E.DIRECT_SMALL = bool(args.direct_small)
    if args.conv1x1 is not None:
        ops.CONV1X1 = bool(args.conv1x1)

    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    # SA_DIST_BACKEND=gloo (and SA_DIST_SHARE_GPU=1): a multi-rank rehearsal of this code path on a
    # single-GPU box (ranks share the GPU; the throughput is then meaningless)
    r = D.init_from_env(os.environ.get("SA_DIST_BACKEND", "nccl"))
    ngpu = torch.cuda.device_count()
    device = torch.device("cuda", r.local_rank % ngpu if os.environ.get("SA_DIST_SHARE_GPU") == "1" else r.local_rank)
    torch.cuda.set_device(device)

    model = StereoAnywhere(dict(PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(device)
    if args.opts:
        import dataclasses
        over = {}
        for kv in args.opts.split(","):
            k_, v_ = kv.split("=")
            cur = getattr(model.opts, k_)
            over[k_] = (v_ not in ("0", "false", "False")) if isinstance(cur, bool) else type(cur)(v_)
        model.opts = dataclasses.replace(model.opts, **over)
    tiled = TILED.get(args.config)
    if tiled is None:
        iters = args.iters or 22
        H, W = args.height, args.width
        Hp, Wp = (H + 31) // 32 * 32, (W + 31) // 32 * 32
        lo, hi = D.shard_range(args.batch * r.world, r.rank, r.world)
        inp = make_inputs(hi - lo, H, W, Hp, Wp, 192.0, seed0=1 + lo, device=device)
        x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])
        runner, units, shape = model, hi - lo, (hi - lo, Hp // 4, Wp // 4)
    else:
        from stereoanywhere_amd import tiler
        from stereoanywhere_amd.offload import CPUOffloadWrapper
        iters = args.iters or tiled["iters"]
        H, W = tiled["image"]
        Hp, Wp = (H + 31) // 32 * 32, (W + 31) // 32 * 32
        # weak scaling over images: every rank tiles its own image
        inp = make_inputs(1, H, W, Hp, Wp, tiled["D"], seed0=1 + r.rank, device=device)
        x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])
        wrap = tiler.from_preset(model, tiled["preset"], batch_tiles=True)
        tiles = wrap._enumerate_tiles(Hp, Wp)
        th, tw = min(wrap.tile_height, Hp), min(wrap.tile_width, Wp)
        # the tiler runs each unique rectangle once (tiler.TileWrapper: duplicates are
        # accumulated again, not recomputed)
        tiled["tiles"], tiled["unique_tiles"], tiled["tile_hw"] = len(tiles), len(set(tiles)), (th, tw)
        # the reference empties the caching allocator after every call (cpu_offload_wrapper.py:82):
        # release_cache=True times that behaviour (--offload-release 0: HBM-resident pools)
        runner = CPUOffloadWrapper(wrap, release_cache=bool(args.offload_release)) if tiled["offload"] else wrap
        units, shape = 1, (len(set(tiles)), th // 4, tw // 4)

    eager_runner = runner
    graph_runner, probe = None, None
    if args.one_stream:
        model.stream_overlap = False
    if tiled is None and not args.no_graph and not args.one_stream:
        # the timed steps replay the whole forward from a hipGraph (inputs copied into its static
        # buffers each step): one host enqueue per forward instead of ~1.4k kernel launches
        from stereoanywhere_amd.graph import ForwardGraph, PipelinedForward
        runner = ForwardGraph(model) if args.pipeline <= 1 else PipelinedForward(model, args.pipeline)

    def step():
        return runner(*x, iters=iters, test_mode=True)

    def eager_step():
        return eager_runner(*x, iters=iters, test_mode=True)

    with torch.no_grad():
        for i in range(args.warmup):
            step()
            torch.cuda.synchronize()
            log(f"warmup {i + 1}/{args.warmup} done")
        # the execution mode for the timed steps, chosen before them: 3 graph replays against 3
        # eager forwards (the same function bit for bit; the replay is usually as fast or
        # faster, but its two-stream overlap has measured 70.3 against 64.9 ms on one box)
        if runner is not eager_runner:
            def _t(fn, n=3):
                torch.cuda.synchronize()
                t_ = time.perf_counter()
                for _ in range(n):
                    fn()
                torch.cuda.synchronize()
                return time.perf_counter() - t_
            t_graph, t_eager = _t(step), _t(eager_step)
            probe = {"graph_ms": t_graph / 3 * 1e3, "eager_ms": t_eager / 3 * 1e3}
            log(f"execution probe: graph {t_graph / 3 * 1e3:.2f} ms, eager {t_eager / 3 * 1e3:.2f} ms per step")
            if t_eager < t_graph:
                graph_runner, runner = runner, eager_runner
                log("timed steps run eagerly (faster on this box)")
        # price the layer-mix-dependent families (Winograd convs, norm epilogues) on one
        # untimed forward
        from stereoanywhere_amd import ops as O
        O.WORK = {}
        eager_step()
        work, O.WORK = O.WORK, None
        torch.cuda.synchronize()
        # timed region: K plain steps -> value.  The per-launch HIP events of the roofline
        # serialise every launch (~6 % of a step), so they run over K more steps right after.
        sysd = _gpu_sysfs(device)
        state_before = box_state(sysd) or {}
        state_before.update(clock_probe(device))
        N.lib().sa_split_redo_blocks(1)   # (synchronises; outside the timed region)
        D.barrier(r)
        torch.cuda.synchronize()
        with BoxSampler(sysd) as sampler:
            t0 = time.perf_counter()
            for _ in range(args.steps):
                out = step()
            torch.cuda.synchronize()
            own = time.perf_counter() - t0   # this rank's own steps (before waiting for the others)
            D.barrier(r)
            elapsed = time.perf_counter() - t0
        redo_blocks = int(N.lib().sa_split_redo_blocks(1))
        state_after = box_state(sysd) or {}
        state_after.update(clock_probe(device))
        log(f"timed {args.steps} steps in {elapsed:.3f} s")
        # cfg5: the other CPUOffloadWrapper cache policy over the same steps (the reference empties the
        # allocator cache after every call, cpu_offload_wrapper.py:82)
        other_release = None
        if tiled is not None and tiled["offload"]:
            runner.release_cache = not runner.release_cache
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            other_release = {"release_cache": runner.release_cache,
                             "ms_per_step": (time.perf_counter() - t4) / args.steps * 1e3}
            runner.release_cache = not runner.release_cache
            log(f"release_cache={other_release['release_cache']}: {other_release['ms_per_step']:.1f} ms/step")
        # the same steps launched eagerly (no graph), for the record (or, when the probe chose
        # eager steps, replayed from the graph)
        other = graph_runner if graph_runner is not None else eager_runner
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for _ in range(args.steps):
            out_e = other(*x, iters=iters, test_mode=True)
        torch.cuda.synchronize()
        elapsed_other = time.perf_counter() - t3
        elapsed_eager = elapsed if runner is eager_runner else elapsed_other
        graph_dev = None
        if runner is not other:   # the replayed forward is the eager one
            graph_dev = float((out[0] - out_e[0]).abs().max())
            if graph_dev != 0.0:
                raise SystemExit(f"bench: the hipGraph replay differs from the eager forward by {graph_dev:g} "
                                 "(it must compute the same function bit for bit); no throughput reported")
        # one-stream plain steps: the schedule the per-launch times below are measured in.  One
        # untimed step first: the whole batch per launch is a new set of shapes (allocator
        # growth, MIOpen kernels built on first use: cfg5's first one-stream steps ran 2.7x slow)
        model.stream_overlap = False
        eager_step()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        one_stream_steps = []
        for _ in range(args.steps):
            ts = time.perf_counter()
            eager_step()
            torch.cuda.synchronize()
            one_stream_steps.append((time.perf_counter() - ts) * 1e3)
        elapsed_1s = time.perf_counter() - t2
        log("one-stream steps (ms): " + ", ".join(f"{v:.1f}" for v in one_stream_steps))
        # per-launch times of one kernel at a time: the side streams' overlap (model.py) would
        # stretch each launch by the work running beside it
        N.timing_enable(True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            eager_step()
        torch.cuda.synchronize()
        elapsed_ev = time.perf_counter() - t1
        kt = {k: N.timing_read(k) for k in N.KERNEL_IDS}
        N.timing_enable(False)
        model.stream_overlap = not args.one_stream
        log(f"instrumented {args.steps} steps in {elapsed_ev:.3f} s")
        per_rank = D.gather_scalars(own, r, device)
        elapsed = D.max_over_ranks(elapsed, r, device)
        # per-unit metrics gathered once, after the timed region (the only data-path collective)
        disp = out[0] if isinstance(out, tuple) else out
        disp = -disp[:, 0] if tiled is None else disp[:, 0]
        local = torch.stack([disp.mean((1, 2)), disp.amin((1, 2)), disp.amax((1, 2))], 1).double()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        allm = D.gather_metrics(local, r)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3

    total_units = units * r.world * args.steps
    if not r.is_main:
        return
    # every hand-written kernel family: algorithmic work / live event time vs MI355X peak
    costs = step_costs(shape[0], shape[1], shape[2], iters)
    costs["conv2d_wino"] = ("TFLOP/s", work.get("conv2d_wino", 0.0))
    costs["conv2d_wino4"] = ("TFLOP/s", work.get("conv2d_wino4", 0.0))
    costs["conv2d_direct"] = ("TFLOP/s", work.get("conv2d_direct", 0.0))
    costs["norm_act"] = ("GB/s", work.get("norm_act", 0.0))
    # the separate GRU gate kernels run only at levels whose width keeps the gates out of the
    # F(4x4) epilogues (W % 4 != 0): priced per call (ops.gru_zr / gru_out, 9 resp. 6-7 planes)
    costs["gru_zr"] = ("GB/s", work.get("gru_zr", 0.0))
    costs["gru_out"] = ("GB/s", work.get("gru_out", 0.0))
    # the update loop's plumbing (pool2x / interp / flow_update: planes read and written once),
    # flow_head.conv2 (256 -> 2 planes), the mono pyramid (volume read, levels written) and convf1
    # (7x7, 2 -> 64 channels on fp32 MFMA), each priced per call (ops._account)
    for k_, u_ in (("gru_plumbing", "GB/s"), ("conv2d_narrow", "GB/s"), ("mono_pyramid", "GB/s"), ("conv1x1", "GB/s"),
                   ("conv2d_small", "TFLOP/s")):
        costs[k_] = (u_, work.get(k_, 0.0))
    kernels = {}
    for k, (ms_tot, n_launch) in kt.items():
        if n_launch == 0 or k not in costs:
            continue
        unit, amount = costs[k]
        secs = ms_tot / 1e3 / args.steps                      # per step
        if unit == "TFLOP/s":
            ach, peak, bound = amount / secs / 1e12, FP32_MFMA_PEAK_TFS, "mfma"
            split4 = (k == "conv2d_wino4" and ops.W4_SPLIT) or (k == "conv2d_direct" and ops.DIRECT_SPLIT)
        else:
            ach, peak, bound = amount / secs / 1e9, HBM_PEAK_GBS, "hbm"
            split4 = False
        kernels[k] = {"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak,
                      "ms_per_step": ms_tot / args.steps, "launches_per_step": n_launch / args.steps,
                      "avg_launch_us": ms_tot * 1e3 / n_launch}
        if split4:
            # the split kernels' fp32 products (path type, peak 157.3 TF/s from the guide) also against
            # the 16x16x16 f16 form's fp32-product rate (2x, self-derived) and as issued f16 flops (4
            # f16 products per fp32 one) against the F16 dense peak (~2.5 PF)
            kernels[k].update(split_peak=SPLIT_MFMA_PEAK_TFS, frac_split_peak=ach / SPLIT_MFMA_PEAK_TFS,
                              f16_issued_tflops=4 * ach, frac_f16_dense_peak=4 * ach / F16_DENSE_PEAK_TFS)
    dom = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
    roof = dict(kernels[dom])
    roof.update({"kernel": dom, "traffic": pmc_traffic(dom, args.batch) if tiled is None else None,
                 "kernels": kernels, "misc_ms_per_step": kt["misc"][0] / args.steps,
                 "schedule": "one-stream (model.stream_overlap = False)",
                 "one_stream_ms_per_step": elapsed_1s / args.steps * 1e3,
                 "one_stream_step_ms": one_stream_steps,
                 "instrumented_ms_per_step": elapsed_ev / args.steps * 1e3,
                 "note": "achieved = algorithmic amount per launch / mean live HIP-event launch time, "
                         "events recorded around every launch over K steps run right after the K "
                         "plain timed steps (the events cost ~6 % of a step), in the one-stream order "
                         "(model.stream_overlap = False, the whole batch per launch; its plain time is "
                         "one_stream_ms_per_step; the headline steps overlap the mono branch and the "
                         "context encoder with the feature encoder on side streams and run the GRU loop "
                         "as two batch parts on two streams, replayed from a hipGraph); "
                         "conv3d_fused counts the direct 3x3x3 convolutions' flops (its stride-1 "
                         "convs execute half of them: F(4,3) Winograd along D); "
                         "fp32 FMA peak 157.3 TF/s is the same for MFMA (v_mfma_f32_*_f32) and VALU; "
                         "conv2d_wino / conv2d_wino4 count the Winograd-domain products they execute "
                         "(16/36 resp. 36/144 of the direct convolution's), so their direct-equivalent "
                         "rates are 2.25x resp. 4x achieved"
                         + ("; conv2d_wino4 / conv2d_direct run the split kernels (ops.W4_SPLIT, "
                            "ops.DIRECT_SPLIT): achieved = their fp32 products (exact f16 hi/lo pair "
                            "products) against the guide's fp32 matrix peak 157.3 TF/s; split_peak "
                            "(2x, the 16x16x16 f16 form) and the issued f16 flops vs the F16 dense peak "
                            "are side fields" if ops.W4_SPLIT or ops.DIRECT_SPLIT else "")
})
    if tiled is None:
        metric, unit = "stereo pairs/sec @540x960 D=192 (1/2/4/8 GPU) + EPE vs reference", "pairs/s"
        if args.config == "cfg4":
            wl = (f"configs[3]: batch {args.batch * r.world} = {args.batch} pairs/GPU x {r.world} GPU"
                  + ("" if r.world == 8 else f" (configs[3]'s per-rank workload; its batch 64 needs 8 GPUs)")
                  + f", {H}x{W} (padded {Hp}x{Wp}), {iters} GRU iters, published flags")
        else:
            wl = (f"configs[1]: batch {args.batch}/GPU x {H}x{W} (padded {Hp}x{Wp}), "
                  f"{iters} GRU iters, published flags")
        config = {"workload": wl, "global_batch": args.batch * r.world,
                  "iters": iters, "parallelism": f"dp{r.world} (independent pairs, metrics all_gather)"}
    else:
        metric, unit = f"stereo images/sec, tiled ({args.config}) + EPE vs reference", "images/s"
        config = {"workload": f"configs[{tiled['index']}]: 1 image/GPU {H}x{W} (padded {Hp}x{Wp}), preset "
                              f"{tiled['preset']} -> {tiled['tiles']} tiles of {th}x{tw} ({tiled['unique_tiles']} unique rectangles, "
                              f"each run once; batch_tiles), "
                              f"{iters} GRU iters, published flags"
                              + (f", CPUOffloadWrapper (HBM-resident weights and mono maps, release_cache="
                                 f"{bool(args.offload_release)})" if tiled["offload"] else ""),
                  "global_batch": r.world, "tiles_per_image": tiled["tiles"],
                  "unique_tile_forwards_per_image": tiled["unique_tiles"], "iters": iters,
                  "release_cache": bool(args.offload_release) if tiled["offload"] else None,
                  "parallelism": f"dp{r.world} (independent images)"}
    res = {
        "metric": metric, "value": total_units / elapsed, "unit": unit, "n_gpus": r.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": ("f32 (" + " and ".join(n for n, on in (("F(4x4) Winograd-domain", ops.W4_SPLIT),
                                                         ("direct-conv", ops.DIRECT_SPLIT)) if on)
                  + " products as exact f16 hi/lo pair products on MFMA, fp32 accumulation; everything else "
                  "fp32)" if ops.W4_SPLIT or ops.DIRECT_SPLIT else "f32"), "data": "synthetic (seeded value-noise pairs, "
        "seeded random weights; no dataset/checkpoint offline)",
        "config": config, "roofline": roof, "gathered_units": int(allm.shape[0]),
        "execution": ("eager launches, chosen over hipGraph replay by the untimed execution probe"
                      if graph_runner is not None else
                      "hipGraph replay of the whole forward (stereoanywhere_amd.graph.ForwardGraph; inputs "
                      "copied into its static buffers each step)" if graph_dev is not None else "eager launches"),
        "eager_ms_per_step": elapsed_eager / args.steps * 1e3,
        "execution_probe": probe,
        # split-kernel blocks the f16 range guard recomputed on fp32 MFMA during the timed steps
        "split_redo_blocks": redo_blocks,
        "split_guard": bool(ops.SPLIT_GUARD),
        "schedule_overrides": args.opts or None,
        "box_state": {"before": state_before, "during": sampler.summary(), "after": state_after},
    }
    if graph_dev is not None:
        res["graph_vs_eager_max_abs"] = graph_dev
    if tiled is not None:
        if other_release is not None:
            res["offload_other_release_cache"] = other_release
        res["tiles_per_s"] = total_units * tiled["tiles"] / elapsed
        res["unique_tile_forwards_per_s"] = total_units * tiled["unique_tiles"] / elapsed
    if not args.no_epe:
        res["epe_vs_reference"] = (epe_vs_reference(model, device) if tiled is None
                                   else epe_vs_reference_tiled(model, device, args.config))
        log(f"EPE vs reference {res['epe_vs_reference']:.3g}")
    if r.world > 1:
        res["rank_timing"] = rank_report(per_rank, args.steps, gather_ms, allm.numel() * 8,
                                         os.environ.get("SA_DIST_BACKEND", "nccl"))
    if not args.no_cpu_baseline:   # (rank 0, after every collective: the other ranks are not held)
        log("cpu baseline (oracle, bounded sample) ...")
        res["cpu_baseline"] = cpu_baseline(iters, Hp, Wp) if tiled is None else cpu_baseline_tile(tiled, iters)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
