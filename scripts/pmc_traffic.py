"""Per-launch HBM traffic of each hand-written kernel family from two rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE, separate runs as MI355X_MICROARCH.md §HBM prescribes).

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced stream, so reads are doubled (the guide's correction; it is exact only for
16-B-per-lane streams, and an upper bound for narrower access).
usage: python scripts/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> out.json
"""
import collections
import csv
import json
import sys

FAMILIES = {
    "conv3d_kernel": "conv3d_fused", "pointwise_upcat_kernel": "conv3d_fused", "pointwise_kernel": "conv3d_fused",
    "conv3d_wd_kernel": "conv3d_fused", "conv3d_onehot_s2_kernel": "conv3d_fused",
    "vol_apply_kernel": "conv3d_fused", "lookup_kernel": "corr_lookup", "lookup_c1_kernel": "corr_lookup", "lookup_c1_vec_kernel": "corr_lookup",
    "corr_pyramid_kernel": "corr_volume_pyramid", "corr_pyramid_v2_kernel": "corr_volume_pyramid", "masked_volume_kernel": "mono_masked_volume",
    "sam_contig_kernel": "softargmin_conf", "sam_strided_kernel": "softargmin_conf", "sam_row_kernel": "softargmin_conf",
    "sam_col_kernel": "softargmin_conf", "sam_slice_kernel": "softargmin_conf",
    "lookup_c1_shear_kernel": "corr_lookup", "shear_kernel": "corr_lookup", "wino_f4k3_persist_kernel": "conv2d_wino4", "lsq_kernel": "weighted_lsq", "lsq_hist_kernel": "weighted_lsq",
    "lsq_solve_kernel": "weighted_lsq",
    "gru_zr_kernel": "gru_zr", "gru_out_kernel": "gru_out", "convex_up_kernel": "convex_upsample",
    "wino_f2k3_kernel": "conv2d_wino", "wino_f4k3_kernel": "conv2d_wino4", "conv_direct_kernel": "conv2d_direct", "norm_act_kernel": "norm_act", "plane_stats_kernel": "norm_act",
    # round 4: the families bench.py times separately (were "misc")
    "pyramid_from_volume_kernel": "mono_pyramid", "pyramid_from_strided_kernel": "mono_pyramid",
    "pool2x_kernel": "gru_plumbing", "pool2x_v4_kernel": "gru_plumbing", "interp_kernel": "gru_plumbing",
    "pool2x_flat_kernel": "gru_plumbing", "interp_flat_kernel": "gru_plumbing", "interp_band_kernel": "gru_plumbing", "resample_multi_kernel": "gru_plumbing",
    "interp_v4_kernel": "gru_plumbing", "flow_update_kernel": "gru_plumbing", "relu_copy_kernel": "gru_plumbing",
    "flow_head_reduce_kernel": "gru_plumbing",
    "conv2d_k3_narrow_kernel": "conv2d_narrow", "conv2d_f1_mfma_kernel": "conv2d_small", "conv2d_small_kernel": "conv2d_small",
    # round 5: the 3-D split-f16 MFMA conv and the implicit-GEMM 3x3 conv
    "conv3d_mf_kernel": "conv3d_fused",
    # the sheared layout's producers and the block-spread lookup
    "lookup_c1_shear_lds_kernel": "corr_lookup", "pyramid_from_strided_sheared_kernel": "mono_pyramid",
    # round 6: the one-launch LSQ, the pixel-per-thread convex upsampling, the split 1x1 GEMM, the
    # stride-2 3-D MFMA conv, the tiler's gather / stitch
    "lsq1_kernel": "weighted_lsq", "convex_up_px_kernel": "convex_upsample", "conv1x1_kernel": "conv1x1",
    "conv1x1_weights_kernel": "conv1x1", "conv3d_s2mf_kernel": "conv3d_fused",
    "tile_gather_pad_kernel": "misc", "tile_stitch_kernel": "misc",
    # round 6 (late): the all-channel 1x1 form, the native feature gates (accounted as misc)
    "conv1x1_v2_kernel": "conv1x1", "feature_gate_stats_kernel": "misc", "feature_gate_apply_kernel": "misc",
}


def family(name):
    for k, v in FAMILIES.items():
        if k in name:
            return v
    return None


def per_launch(path, counter):
    tot = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        f = family(r["Kernel_Name"])
        if f:
            tot[f] += float(r["Counter_Value"])
            n[f].add(r["Dispatch_Id"])
    return {f: tot[f] * 1024.0 / len(n[f]) for f in tot}


if __name__ == "__main__":
    fetch = per_launch(sys.argv[1], "FETCH_SIZE")
    write = per_launch(sys.argv[2], "WRITE_SIZE")
    out = {f: {"fetch_bytes_raw": fetch.get(f), "write_bytes": write.get(f),
               "hbm_bytes_per_launch": 2.0 * fetch.get(f, 0.0) + write.get(f, 0.0)} for f in set(fetch) | set(write)}
    json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))
