#!/usr/bin/env python3
"""Throughput of the MI355X StereoAnywhere forward on synthetic 540x960 pairs.

    python bench.py [--gpus N --steps K --warmup W]
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
                reference) on one 544x960 pair, all host threads, N=1 only
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
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

PUBLISHED = dict(use_truncate_vol=True, use_aggregate_mono_vol=True, vol_n_masks=8, n_additional_hourglass=0,
                 vol_downsample=0, mirror_conf_th=0.98, mirror_attenuation=0.9, lrc_th=1.0, normal_gain=10)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8 TB/s spec
FP32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_*_f32 dense peak


def step_costs(B: int, H4: int, W4: int, iters: int, C: int = 256):
    """Algorithmic work of one forward step per hand-written kernel family:
    {kernel: (unit, amount per step)} — minimal bytes each launch must move (HBM-bound
    kernels) or flops it must do (compute-bound ones).  Derivations in DESIGN.md §4."""
    px = B * H4 * W4                      # 1/4-res pixels
    vol = px * W4                         # cost-volume cells
    lv = [W4 >> i for i in range(4)]
    gru_px = B * (H4 * W4 + ((H4 + 1) // 2) * ((W4 + 1) // 2) + ((H4 + 3) // 4) * ((W4 + 3) // 4))
    hid = 128
    return {
        # fp32 MFMA: 2*C flops per volume cell (a1); epilogue work (trunc, pyramid) is free
        "corr_volume_pyramid": ("TFLOP/s", 2.0 * vol * C),
        # per pixel: 2 volumes x 4 levels x (2r+2) cells read, coords read, and (convc1 fused)
        # 2 x 64 channels of relu(convc1(taps)) written
        "corr_lookup": ("GB/s", iters * px * (2 * 4 * 10 * 4 + 4 + 2 * 64 * 4)),
        "mono_masked_volume": ("GB/s", 8 * vol * 4 + px * 2 * 4 * 4),
        # two aggregated volumes read once, four maps written
        "softargmin_conf": ("GB/s", 2 * vol * 4 + 4 * px * 4),
        # three joint L/R maps read once
        "weighted_lsq": ("GB/s", 3 * 2 * px * 4),
        # per pixel and GRU level: xc(2C) + hzr(2C) + cz,cr(2C) + h(C) read, z, r*h (2C) written
        "gru_zr": ("GB/s", iters * gru_px * 9 * hid * 4),
        # xc_q, qh, cq, z, h read, h written
        "gru_out": ("GB/s", iters * gru_px * 6 * hid * 4),
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


def make_inputs(B, H, W, Hp, Wp, D, seed0, device):
    pb = synth.synthetic_batch(B, H, W, D, seed0=seed0)
    out = {}
    for k in ("left", "right", "mono_left", "mono_right"):
        x, _ = synth.pad_to_multiple(pb[k], 32)
        assert x.shape[-2:] == (Hp, Wp)
        out[k] = torch.from_numpy(np.ascontiguousarray(x)).to(device)
    return out


def host_threads() -> int:
    """CPU share of this process: OMP_NUM_THREADS if set (16 on the GPU box), else the
    affinity mask — os.cpu_count() reports the whole machine there."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(iters: int, H: int, W: int):
    """The oracle restatement on one pair (bounded sample), all host threads."""
    from oracle import model_ref as M

    torch.set_num_threads(host_threads())
    sd = M.load_state_dict_seeded(0)
    pair = synth.synthetic_batch(1, H, W, 192.0, seed0=1)
    t = [torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")]
    t0 = time.perf_counter()
    M.forward(sd, *t, iters=iters)
    dt = time.perf_counter() - t0
    return {"value": 1.0 / dt, "unit": "pairs/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"1 pair 1x{H}x{W}, {iters} iters, oracle (torch CPU convs + numpy hot path), "
                      f"{dt:.1f} s wall"}


def epe_vs_reference(model, device):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_util import load_fixture, regenerate_inputs  # golden data only

    fix = load_fixture("cfg2_544x960_it22.npz")
    pair = regenerate_inputs(fix, 1, 544, 960, 192.0)
    t = [torch.from_numpy(pair[k]).to(device) for k in ("left", "right", "mono_left", "mono_right")]
    flow_up, _ = model(*t, iters=22, test_mode=True)
    disp = -flow_up[:, 0].cpu().numpy()
    return float(np.abs(disp.astype(np.float64) - fix["disparity"]).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4, help="pairs per GPU (configs[1]: 4)")
    ap.add_argument("--iters", type=int, default=22)
    ap.add_argument("--height", type=int, default=540)
    ap.add_argument("--width", type=int, default=960)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-epe", action="store_true")
    ap.add_argument("--miopen-find", type=int, default=0,
                    help="let MIOpen time its conv algorithms per shape (torch cudnn.benchmark)")
    args = ap.parse_args()

    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    r = D.init_from_env("nccl")
    device = torch.device("cuda", r.local_rank)
    torch.cuda.set_device(device)
    if r.world != args.gpus and r.is_main:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {r.world}", file=sys.stderr)

    H, W = args.height, args.width
    Hp, Wp = (H + 31) // 32 * 32, (W + 31) // 32 * 32
    H4, W4 = Hp // 4, Wp // 4
    model = StereoAnywhere(dict(PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(device)
    lo, hi = D.shard_range(args.batch * r.world, r.rank, r.world)
    inp = make_inputs(hi - lo, H, W, Hp, Wp, 192.0, seed0=1 + lo, device=device)
    x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])

    with torch.no_grad():
        for i in range(args.warmup):
            model(*x, iters=args.iters, test_mode=True)
            torch.cuda.synchronize()
            log(f"warmup {i + 1}/{args.warmup} done")
        # price the layer-mix-dependent families (Winograd convs, norm epilogues) on one
        # untimed forward
        from stereoanywhere_amd import ops as O
        O.WORK = {}
        model(*x, iters=args.iters, test_mode=True)
        work, O.WORK = O.WORK, None
        torch.cuda.synchronize()
        # timed region: K plain steps -> value.  The per-launch HIP events of the roofline
        # serialise every launch (~6 % of a step), so they run over K more steps right after.
        D.barrier(r)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out, _ = model(*x, iters=args.iters, test_mode=True)
        torch.cuda.synchronize()
        D.barrier(r)
        elapsed = time.perf_counter() - t0
        log(f"timed {args.steps} steps in {elapsed:.3f} s")
        # per-launch times of one kernel at a time: the side streams' overlap (model.py) would
        # stretch each launch by the work running beside it
        model.stream_overlap = False
        N.timing_enable(True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            model(*x, iters=args.iters, test_mode=True)
        torch.cuda.synchronize()
        elapsed_ev = time.perf_counter() - t1
        kt = {k: N.timing_read(k) for k in N.KERNEL_IDS}
        N.timing_enable(False)
        model.stream_overlap = True
        log(f"instrumented {args.steps} steps in {elapsed_ev:.3f} s")
        elapsed = D.max_over_ranks(elapsed, r, device)
        # per-pair metrics gathered once, after the timed region (the only collective)
        disp = -out[:, 0]
        local = torch.stack([disp.mean((1, 2)), disp.amin((1, 2)), disp.amax((1, 2))], 1).double()
        allm = D.gather_metrics(local, r)

    total_pairs = args.batch * r.world * args.steps
    if not r.is_main:
        return
    # every hand-written kernel family: algorithmic work / live event time vs MI355X peak
    costs = step_costs(hi - lo, H4, W4, args.iters)
    costs["conv2d_wino"] = ("TFLOP/s", work.get("conv2d_wino", 0.0))
    costs["conv2d_wino4"] = ("TFLOP/s", work.get("conv2d_wino4", 0.0))
    costs["conv2d_direct"] = ("TFLOP/s", work.get("conv2d_direct", 0.0))
    costs["norm_act"] = ("GB/s", work.get("norm_act", 0.0))
    kernels = {}
    for k, (ms_tot, n_launch) in kt.items():
        if n_launch == 0 or k not in costs:
            continue
        unit, amount = costs[k]
        secs = ms_tot / 1e3 / args.steps                      # per step
        if unit == "TFLOP/s":
            ach, peak, bound = amount / secs / 1e12, FP32_MFMA_PEAK_TFS, "mfma"
        else:
            ach, peak, bound = amount / secs / 1e9, HBM_PEAK_GBS, "hbm"
        kernels[k] = {"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak,
                      "ms_per_step": ms_tot / args.steps, "launches_per_step": n_launch / args.steps,
                      "avg_launch_us": ms_tot * 1e3 / n_launch}
    dom = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
    roof = dict(kernels[dom])
    roof.update({"kernel": dom, "traffic": pmc_traffic(dom, args.batch), "kernels": kernels,
                 "misc_ms_per_step": kt["misc"][0] / args.steps,
                 "instrumented_ms_per_step": elapsed_ev / args.steps * 1e3,
                 "note": "achieved = algorithmic amount per launch / mean live HIP-event launch time, "
                         "events recorded around every launch over K steps run right after the K "
                         "plain timed steps (the events cost ~6 % of a step), in the one-stream order "
                         "(model.stream_overlap = False: the plain steps overlap the mono branch and the "
                         "context encoder with the feature encoder on side streams); "
                         "fp32 FMA peak 157.3 TF/s is the same for MFMA (v_mfma_f32_*_f32) and VALU; "
                         "conv2d_wino / conv2d_wino4 count the Winograd-domain products they execute "
                         "(16/36 resp. 36/144 of the direct convolution's), so their direct-equivalent "
                         "rates are 2.25x resp. 4x achieved"})
    res = {
        "metric": "stereo pairs/sec @540x960 D=192 (1/2/4/8 GPU) + EPE vs reference",
        "value": total_pairs / elapsed, "unit": "pairs/s", "n_gpus": r.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded value-noise pairs, "
        "seeded random weights; no dataset/checkpoint offline)",
        "config": {"workload": f"configs[1]: batch {args.batch}/GPU x {H}x{W} (padded {Hp}x{Wp}), "
                               f"{args.iters} GRU iters, published flags", "global_batch": args.batch * r.world,
                   "iters": args.iters, "parallelism": f"dp{r.world} (independent pairs, metrics all_gather)"},
        "roofline": roof,
        "gathered_pairs": int(allm.shape[0]),
    }
    if not args.no_epe:
        res["epe_vs_reference"] = epe_vs_reference(model, device)
        log(f"EPE vs reference {res['epe_vs_reference']:.3g}")
    if r.world == 1 and not args.no_cpu_baseline:
        log("cpu baseline (oracle, bounded sample) ...")
        res["cpu_baseline"] = cpu_baseline(args.iters, Hp, Wp)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
