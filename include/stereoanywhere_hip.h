/*
 * stereoanywhere_hip.h — C ABI of the MI355X (gfx950) cost-volume hot path.
 *
 * One shared library, libsa_hip.so, built by hipcc from the .hip sources in
 * stereoanywhere_amd/csrc/.
 * Every entry point takes plain device pointers and sizes (no framework types):
 *   - all tensors are float32, dense, row-major in the layout documented per call;
 *   - `stream` is a hipStream_t (NULL = the default stream); calls only enqueue work
 *     and never synchronise the host (the reference's implicit syncs at
 *     utils/utils.py:26 and :361-368 disappear);
 *   - the return value is SA_OK or a negative SA_E_* code; sa_last_error() gives a
 *     message for the calling thread.  Argument checks reproduce the failures the
 *     reference raises as Python exceptions (stereoanywhere.py:133, utils.py:26).
 *
 * The library replaces the torch-level operator plug-in point of the reference:
 * `args.corr_implementation` (stereoanywhere.py:25, 128-133) and the `CorrBlock1D`
 * class contract (corr.py:75-132) — see INTEGRATION.md for the bindings.
 * Reference paths below are relative to the kei312/stereoanywhere root.
 */
#ifndef STEREOANYWHERE_HIP_H
#define STEREOANYWHERE_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header.  Bumped whenever an entry point's signature or a struct passed by
 * pointer or in an array changes (INTEGRATION.md lists the breaks).  A host checks at load time
 * that sa_abi_version() == SA_ABI_VERSION and that sa_struct_size(SA_STRUCT_*) equals its own
 * sizeof: the arrays of SaWinoProblem / SaGateEpilogue / SaResampleJob are read at the library's
 * stride, so a host built against another layout would hand over misread fields.
 *   7: sa_feature_gates / SaFeatureGateJob added (additive: no earlier entry point changed)
 *   6: round 6 (the implicit-GEMM entry points removed; sa_struct_size, sa_conv3d_mf_get_planes)
 *   5: SaWinoProblem gained the residual-epilogue fields (skip ... out_act); sa_conv2d_k3_wino4_launch
 *      took a guard flag; sa_conv2d_wino4_weights_cb removed */
#define SA_ABI_VERSION 7
enum { SA_STRUCT_WINO_PROBLEM = 0, SA_STRUCT_GATE_EPILOGUE = 1, SA_STRUCT_RESAMPLE_JOB = 2, SA_STRUCT_FEATURE_GATE_JOB = 3 };
int sa_abi_version(void);
/* sizeof the struct `which` (SA_STRUCT_*) as the library was built, -1 for an unknown id */
long sa_struct_size(int which);

enum {
  SA_OK = 0,
  SA_E_ARG = -1,        /* bad shape / null pointer / unsupported size           */
  SA_E_LAUNCH = -2,     /* hipLaunchKernel or hipGetLastError failed             */
  SA_E_RUNTIME = -3     /* other HIP runtime failure (events, memset)            */
};

const char *sa_last_error(void);

/* ----------------------------------------------------------------------------------
 * Correlation pyramid storage.  The reference keeps num_levels+1 separate tensors
 * [B*H*W1, 1, 1, W2>>i] (corr.py:85-91).  Here one buffer holds, for every pixel row
 * (b,h,j), the levels back to back: [L0 (W2) | L1 (W2/2) | L2 | L3 ...] (floor at every
 * halving), the row padded to a multiple of 4 floats.  Level `num_levels` (built but
 * never read by the reference, corr.py:101) is not stored.
 * ---------------------------------------------------------------------------------- */
int  sa_pyramid_level_width(int w2, int level);
int  sa_pyramid_level_offset(int w2, int level);
long sa_pyramid_row_stride(int w2, int num_levels);

/* a1 + a8 + a9 — replaces CorrBlock1D.corr (corr.py:117-132) followed by the
 * truncation multiply (stereoanywhere.py:201-205, 253-254, utils.py:216-238) and
 * CorrBlock1D.__init__ (corr.py:76-91).
 *   fmap2 [B,C,H,W1], fmap3 [B,C,H,W2]  (NCHW, as produced by fnet)
 *   V[b,h,j,k] = sum_c fmap2[b,c,h,j] fmap3[b,c,h,k] / sqrt_c   (fp32 MFMA, exact f32)
 *   if trunc_disp != NULL:  V *= (1 - m) + m (sigmoid((j - d) - k)(1 - atten) + atten)
 *     with d = trunc_disp[b,h,j], m = trunc_conf[b,h,j]   ([B,H,W1] each)
 *   pyramid: [B*H*W1, row_stride] as above, levels 0..num_levels-1 written.
 * num_levels = 1 gives the plain volume ([B,H,W1,W2] when row_stride == W2). */
int sa_corr_volume_pyramid(const float *fmap2, const float *fmap3, int B, int C, int H, int W1,
                           int W2, float sqrt_c, const float *trunc_disp, const float *trunc_conf,
                           float atten, int num_levels, float *pyramid, long row_stride,
                           void *stream);

/* a9 alone — CorrBlock1D.__init__ (corr.py:76-91) on an existing volume.
 *   volume: `rows` rows of W2 floats with stride in_row_stride (level 0 is copied). */
int sa_corr_pyramid_from_volume(const float *volume, long rows, int W2, long in_row_stride,
                                int num_levels, float *pyramid, long row_stride, void *stream);
/* The same pyramid from a volume whose element (b, h, j, k) sits at volume + b*sb + h*sh + j +
 * k*sk (W1 contiguous, any W2, staged in 256-wide chunks: the hourglass's [B, 1, W2, H, W1] classifier output, used as
 * the mono volume with use_aggregate_mono_vol, stereoanywhere.py:168, 210); pyramid rows in
 * (b, h, j) order as above. */
int sa_corr_pyramid_from_volume_strided(const float *volume, int B, int H, int W1, int W2, long sb, long sh, long sk,
                                        int num_levels, float *pyramid, long row_stride, void *stream);

/* a10 — CorrBlock1D.__call__ (corr.py:93-115) + bilinear_sampler (utils.py:19-35).
 *   coords_x: x channel of coords1, element (b,h,j) at coords_x[b*coords_bstride + h*W1 + j]
 *   out: element (b, v*L*(2r+1) + l*(2r+1) + t, h, j) at
 *        out[b*out_bstride + (v*L*(2r+1) + l*(2r+1) + t)*H*W1 + h*W1 + j]
 *   where v = 0 for pyramid_a and 1 for pyramid_b (pyramid_b may be NULL).  Zero
 *   padding outside [0, W_l - 1]; same normalise/unnormalise round trip as grid_sample. */
int sa_corr_lookup(const float *pyramid_a, const float *pyramid_b, int W2, long row_stride,
                   int num_levels, int radius, const float *coords_x, long coords_bstride,
                   int B, int H, int W1, float *out, long out_bstride, void *stream);

/* a2 — estimate_normals (utils.py:73-77) on the 1/4-res mono map.
 *   mde [B,1,H,W] -> normals [B,3,H,W]; gain = W/normal_gain (stereoanywhere.py:113). */
int sa_mono_normals(const float *mde, int B, int H, int W, float gain, float *normals,
                    void *stream);

/* a2 + a3 — 1.73 * corr(normals_l, normals_r) (stereoanywhere.py:136) binned by the
 * half-open depth masks (utils.py:48-54, stereoanywhere.py:138-139, 161), written
 * directly in the hourglass's [B, nbins, W2, H, W1] layout (hourglass.py:63).
 *   n2 [B,3,H,W1], n3 [B,3,H,W2], m2 [B,1,H,W1], m3 [B,1,H,W2] (1/4-res mono maps). */
int sa_mono_masked_volume(const float *n2, const float *n3, const float *m2, const float *m3,
                          int B, int H, int W1, int W2, int nbins, float gain, float *out,
                          void *stream);

/* a2 + a3 without the volume — per-pixel records (n0, n1, n2, bin) of one view (normals of
 * estimate_normals, utils.py:73-77; depth bin of generate_masks, utils.py:48-54, -1 = none):
 *   normals [B,3,H,W], m [B,1,H,W] -> rec [B,H,W] float4 (16-byte aligned).  Masked-volume
 *   cell (n, k, h, j) = gain * (nL[h,j] . nR[h,k]) / sqrt(3) iff binL[h,j] == binR[h,k] == n
 *   (stereoanywhere.py:136, 161): what sa_conv3d_onehot / sa_conv3d_pointwise_upcat_onehot
 *   evaluate in place of reading the [B, nbins, W2, H, W1] volume. */
int sa_mono_bin_records(const float *normals, const float *m, int B, int H, int W, int nbins,
                        float *rec, void *stream);

/* a5 + a6 — estimate_left/right_disparity (utils.py:112-152) and
 * estimate_left/right_confidence (utils.py:154-170) on volumes given by strides
 * (element (b,h,j,k) at v[b*sb + h*sh + j*sj + k*sk]; sj == 1 or sk == 1).
 *   vol_disp -> dL [B,H,W1], dR [B,H,W2];  vol_conf -> cL [B,H,W1], cR [B,H,W2], each
 *   output map's element (b,h,o) at out[b*out_bs + h*W + o] (out_bs = H*W for [B,1,H,W]). */
int sa_softargmin_conf(const float *vol_disp, const float *vol_conf, int B, int H, int W1,
                       int W2, long sb, long sh, long sj, long sk, float *dL, float *dR,
                       float *cL, float *cR, long out_bs, void *stream);
/* With sj == 1 and W1 == W2 <= 288 (the model's layout) sa_softargmin_conf reads each volume
 * once: a workgroup per (b, h) slice forms both sides' reductions.  on = 0 selects the per-line
 * kernels instead (two launches, each reading both volumes), on = 2 the one-pass kernel's
 * 16-byte-row variant (n % 4 == 0, n <= 256, aligned rows; slower); for A/B runs and tests. */
void sa_softargmin_set_one_pass(int on);
int sa_softargmin_get_one_pass(void);

/* a7 — softlrc (utils.py:189-198) with disp_warping (utils.py:172-187); optional
 * fuzzy_and with a confidence (utils.py:240-241, stereoanywhere.py:188-189):
 *   s2 = softlrc_2 * (conf2 ? conf2 : 1), s3 likewise.  All maps [H,W] planes with batch
 *   stride map_bs (H*W for [B,1,H,W]; 2*H*W for the L/R halves of a [B,2,H,W] buffer). */
int sa_softlrc(const float *d2, const float *d3, const float *conf2, const float *conf3, int B,
               int H, int W, long map_bs, float lrc_th, float *s2, float *s3, void *stream);

/* a7 — weighted_lsq (utils.py:345-384) over the joint L+R maps of each sample:
 *   maps [B, 2, H, W] each (mde, disp, conf); exact torch.quantile(linear) band
 *   [q_lo, q_hi] on relu(disp) (radix select, no host sync), weighted least squares in
 *   float64 accumulation.  Writes scale[B], shift[B] (device). */
int sa_weighted_lsq(const float *mde, const float *disp, const float *conf, int B, int n_per_b,
                    float q_lo, float q_hi, float *scale, float *shift, void *stream);

/* a7 — the same result spread over the whole GPU (n_per_b / 2048 blocks per sample, five
 * launches: one per radix digit, then the normal equations).  ws: sa_weighted_lsq_ws_size
 * bytes of device memory, 16-byte aligned, ZEROED before the call (left zeroed after it). */
long sa_weighted_lsq_ws_size(int B, int n_per_b);
int sa_weighted_lsq_ws(const float *mde, const float *disp, const float *conf, int B, int n_per_b,
                       float q_lo, float q_hi, float *scale, float *shift, void *ws, void *stream);

/* a7 + a8 + a11 — scaled mono (stereoanywhere.py:194-197), its softLRC (199), the mirror
 * detector (utils.py:255-269) and the initial coordinates (stereoanywhere.py:261-262):
 *   sm2 = scale*m2 + shift, sm3 = scale*m3 + shift                     [B,1,H,W]
 *   mirror = detector(dL, sm2, conf_l, softlrc(sm2, sm3))              [B,1,H,W]
 *   coords_x = x - sm2                                                  [B,1,H,W]
 * Inputs m2, m3, dL, conf_l are [H,W] planes with batch stride in_bs; outputs dense. */
int sa_mono_scale_mirror(const float *m2, const float *m3, const float *scale, const float *shift,
                         const float *dL, const float *conf_l, int B, int H, int W, long in_bs,
                         float lrc_th, float conf_th, float *sm2, float *sm3, float *mirror,
                         float *coords_x, void *stream);

/* a12 — ConvGRU gates (update.py:53-62) with the convolution split by input
 * (conv([h,x]) = conv_h(h) + conv_x(x)); all tensors [B, ch, H, W] with batch strides.
 *   gru_zr: z = sigmoid(xc[0:C] + hzr[0:C] + cz), r = sigmoid(xc[C:2C] + hzr[C:2C] + cr),
 *           writes z and rh = r*h.
 *   gru_out: h = (1 - z) h + z tanh(xc[2C:3C] + qh + cq)   (in place on h). */
int sa_gru_zr(const float *xc, long xc_bs, const float *bx, const float *hzr, long hzr_bs, const float *cz,
              const float *cr, long c_bs, const float *h, long h_bs, int B, int C, int HW,
              float *z, float *rh, void *stream);
int sa_gru_out(const float *xc, long xc_bs, const float *bx, const float *qh, long qh_bs, const float *cq,
               long c_bs, const float *z, int B, int C, int HW, float *h, long h_bs,
               void *stream);
/* As sa_gru_out with the r*h conv split over its input channels: the gate reads qh + qh2
 * (both with batch stride qh_bs; qh2 may be NULL). */
int sa_gru_out_split(const float *xc, long xc_bs, const float *bx, const float *qh, const float *qh2, long qh_bs,
                     const float *cq, long c_bs, const float *z, int B, int C, int HW, float *h, long h_bs,
                     void *stream);

/* Update-block plumbing that writes straight into channel slices of the GRU inputs
 * (replaces the torch.cat calls of update.py:54-59, 88-90):
 *   pool2x: avg_pool2d(3, stride 2, pad 1, count_include_pad) (update.py:124-125)
 *   interp: bilinear, align_corners=True resize (update.py:130-132)
 *   relu_copy: out = max(in, 0)
 *   flow_update: coords_x += delta[:, 0] (delta may be NULL; stereoanywhere.py:277-280) and
 *     writes the 2-plane flow [coords_x - x, 0] (stereoanywhere.py:272) into flow_a and
 *     flow_b (either may be NULL) — the convf1 input and the tail of the motion
 *     features (update.py:90). */
int sa_pool2x(const float *in, long in_bs, int B, int C, int H, int W, float *out, long out_bs,
              void *stream);
int sa_interp_bilinear_ac(const float *in, long in_bs, int B, int C, int H, int W, int Ho, int Wo,
                          float *out, long out_bs, void *stream);
/* The same on pitched planes ([H][in_pitch] in, [Ho][out_pitch] out; pitch >= width; columns
 * beyond the width are neither read nor written): the padded planes of a GRU level whose width
 * is not a multiple of 4 (SaWinoProblem.pitch). */
int sa_pool2x_p(const float *in, long in_bs, int in_pitch, int B, int C, int H, int W, float *out,
                long out_bs, int out_pitch, void *stream);
int sa_interp_bilinear_ac_p(const float *in, long in_bs, int in_pitch, int B, int C, int H, int W,
                            int Ho, int Wo, float *out, long out_bs, int out_pitch, void *stream);
/* Up to 4 independent pool2x / interp jobs (the pitched forms above) in ONE launch: the update
 * loop's plumbing between two conv launches (update.py:124-132: pool2x(net[0]) and
 * interp(net[2]) feed gru16; interp(net[1]) feeds gru08 and pool2x(net[1]) gru32).  pool2x:
 * (Ho, Wo) must be ((H-1)/2+1, (W-1)/2+1).  Same results as the one-job entry points. */
/* SA_RESAMPLE_FLOW_X: the motion encoder's flow planes from the coordinates, sa_flow_update with
 * only flow_b: in = coords [B,1,H,W] (dense, batch stride in_bs), out = [B,2,H,W] planes (batch
 * stride out_bs): out[0] = coords - x, out[1] = 0; C = 1, (Ho, Wo) = (H, W), pitches = W. */
enum { SA_RESAMPLE_POOL2X = 0, SA_RESAMPLE_BILINEAR_AC = 1, SA_RESAMPLE_FLOW_X = 2 };
typedef struct SaResampleJob {
  int kind;
  const float *in;
  long in_bs;
  int in_pitch;
  int B, C, H, W, Ho, Wo;
  float *out;
  long out_bs;
  int out_pitch;
} SaResampleJob;
int sa_resample_multi(int njobs, const SaResampleJob *jobs, void *stream);

/* a4 — the DoubleFeatureAtt gates of the hourglass (submodule.py:113-140; hourglass.py:66-91): per
 * job and image, out[c] = sigmoid(b1[c] + sum_k w1[c][k] leaky(IN(conv3x3(in, w3[k])))) over 32
 * hidden channels (conv3x3 with zero padding and no bias, InstanceNorm2d without affine, eps 1e-5,
 * biased variance, LeakyReLU 0.01), in a one-channel plane [B][H][W] (image stride in_bs), w3
 * [32][9], w1 [C][32], b1 [C] (NULL: 0), out [B][C][H][W] (image stride out_bs), C <= 64.  Up to
 * SA_GATE_MAX_JOBS jobs in two launches; ws of sa_feature_gates_ws_size bytes (fp64 partial sums,
 * no zeroing needed: every slot is written before it is read). */
#define SA_GATE_MAX_JOBS 8
typedef struct SaFeatureGateJob {
  const float *in;
  long in_bs;
  int B, H, W;
  const float *w3, *w1, *b1;
  int C;
  float *out;
  long out_bs;
} SaFeatureGateJob;
long sa_feature_gates_ws_size(int njobs, const SaFeatureGateJob *jobs);
int sa_feature_gates(int njobs, const SaFeatureGateJob *jobs, void *ws, void *stream);
int sa_relu_copy(const float *in, long in_bs, int B, int C, int HW, float *out, long out_bs,
                 void *stream);
int sa_flow_update(float *coords_x, const float *delta, long delta_bs, int B, int H, int W,
                   float *flow_a, long flow_a_bs, float *flow_b, long flow_b_bs, void *stream);

/* a10 + update.py:75, 84 — the lookup of sa_corr_lookup fused with the motion encoder's convc1
 * (1x1 conv of the L*(2r+1) taps -> Cout, + bias, ReLU): weight_kc [L*(2r+1)][Cout] (the
 * module's [Cout][K][1][1] transposed), out [B*nvol, Cout, H, W1] with sample b*nvol + v
 * (v = 0 for pyramid_a, 1 for pyramid_b).  Built for 4 levels, radius 4, Cout 64. */
int sa_corr_lookup_conv1x1(const float *pyramid_a, const float *pyramid_b, int W2, long row_stride,
                           int num_levels, int radius, const float *coords_x, long coords_bstride,
                           int B, int H, int W1, const float *weight_kc, const float *bias, int Cout,
                           float *out, void *stream);
/* a10 on a disparity-sheared pyramid (csrc/corr_shear.hip): level l of image row (b, h) as
 * S_l[e][j] = C_l[j][(j >> l) - e + W_l - 1], e in [0, W_l + ((W1 - 1) >> l)), rows
 * sa_shear_row_pitch(W1) = W1 rounded up to 32 floats apart (whole 128-byte lines per 32-pixel
 * segment), levels back to back at sa_shear_level_offset in a slice of sa_shear_slice_size floats
 * per image row: a wave's neighbouring pixels then read neighbouring addresses.  Cells whose k = (j >> l) - e + W_l - 1 falls outside [0, W_l) are not
 * written (the lookup's tap test gives the reference's zero padding there without using them).
 *   sa_corr_pyramid_shear: the row-layout pyramid [B*H*W1][row_stride] -> sheared [B*H][slice]
 *   sa_corr_volume_pyramid_sheared: sa_corr_volume_pyramid written sheared (C % 16 == 0, W1 and
 *     W2 % 4 == 0, 16-byte aligned feature maps under 2 GiB; the same cell values)
 *   sa_corr_pyramid_from_volume_strided_sheared: sa_corr_pyramid_from_volume_strided written
 *     sheared
 *   sa_corr_lookup_conv1x1_sheared: sa_corr_lookup_conv1x1 on sheared pyramids (same taps,
 *     same arithmetic; 4 levels, radius 4, Cout 64). */
/* convc1 of the fused lookups (both layouts) on the VALU (0, default) or fp32 MFMA (1, measured
 * slower): the same k-ordered fmaf chain either way.  For A/B runs and tests. */
void sa_lookup_set_mfma(int on);
int sa_lookup_get_mfma(void);
/* the sheared lookup's work split: 3 (default) / 2 spread over an 8 / 4-wave block per 64 pixels
 * (a thread per (pixel, volume, level) gathers the taps into LDS, then a thread per (pixel, channel
 * group) runs convc1), 1 both volumes in one thread, 0 one volume per thread.  A/B and tests. */
void sa_lookup_set_shear_dual(int on);
int sa_lookup_get_shear_dual(void);
long sa_shear_slice_size(int W1, int W2, int num_levels);
long sa_shear_row_pitch(int W1);
/* 1 when sa_corr_pyramid_shear + sa_corr_lookup_conv1x1_sheared take this geometry (B*H <= 65535,
 * W2 <= 511, 4 levels with the coarsest >= 2 wide), else 0: the caller keeps the row layout */
int sa_corr_shear_supported(int B, int H, int W1, int W2, int num_levels);
long sa_shear_level_offset(int W1, int W2, int num_levels, int level);
int sa_corr_pyramid_shear(const float *pyramid, long row_stride, int B, int H, int W1, int W2,
                          int num_levels, float *sheared, void *stream);
int sa_corr_volume_pyramid_sheared(const float *fmap2, const float *fmap3, int B, int C, int H, int W1,
                                   int W2, float sqrt_c, const float *trunc_disp,
                                   const float *trunc_conf, float atten, int num_levels,
                                   float *sheared, void *stream);
int sa_corr_pyramid_from_volume_strided_sheared(const float *volume, int B, int H, int W1, int W2,
                                                long sb, long sh, long sk, int num_levels,
                                                float *sheared, void *stream);
int sa_corr_lookup_conv1x1_sheared(const float *sheared_a, const float *sheared_b, int W2,
                                   int num_levels, int radius, const float *coords_x,
                                   long coords_bstride, int B, int H, int W1,
                                   const float *weight_kc, const float *bias, int Cout,
                                   float *out, void *stream);

/* a14 — convex_upflow (utils.py:97-110), factor 4: flow [B,1,H,W] (low-res x flow),
 * mask [B, 9*f*f, H, W] -> out [B,1,f*H,f*W] (sign as given: the reference's
 * flow_up, i.e. minus the disparity). */
int sa_convex_upsample(const float *flow, const float *mask, long mask_bs, int B, int H, int W,
                       int factor, float *out, void *stream);

/* Mono hourglass (hourglass.py:13-91, submodule.py:25-53, 113-140) and its classifiers
 * (stereoanywhere.py:165-166) as fused direct 3-D convolutions on [B, C, D, H, W] volumes
 * (D = W2, W = W1), 3x3x3 / pad 1 / no bias, stride 1 or 2:
 *   out = conv(T(in)),  T(x) = [gate_l[b,c,h,w] * gate_r[b,c,h,d] *] [lrelu(] [(x - mean[b,c]) *
 *   rstd[b,c]] [)] — the previous layer's InstanceNorm3d + LeakyReLU (+ DoubleFeatureAtt
 *   gate, maps at the INPUT resolution) applied while the input is staged.
 *   stats_partial (may be NULL): per-block float64 (sum, sum^2) of every output channel,
 *   [B*Cout][parts][2] with parts = sa_conv3d_stat_parts(Cout, stride, Do, Ho, Wo);
 *   reduce with sa_instnorm_finalize.  Output size (n - 1) / stride + 1 per axis.
 * Built for (Cin, Cout, stride) in {(8,8,1), (8,2,1), (16,16,1), (32,32,1), (8,16,2), (16,32,2)}. */
long sa_conv3d_stat_parts(int Cout, int stride, int Do, int Ho, int Wo);
int sa_conv3d(const float *in, int B, int Cin, int Di, int Hi, int Wi, int stride,
              const float *weight, int Cout, const float *in_mean, const float *in_rstd, int act,
              float slope, const float *gate_l, const float *gate_r, float *out,
              double *stats_partial, void *stream);
/* 1x1x1 conv over cat(Ta(a), trilinear_up(T(u))) (hourglass.py:319-321, 326-328), in two
 * launches because the upsample is linear: W . cat(Ta(a), up(T(u))) = Wa . Ta(a) + up(Wu . T(u)).
 *   sa_conv3d_pointwise: p = W . T(in) at the low resolution (transform T as for sa_conv3d,
 *     weight [Cin][Cout]; no statistics).  Built for 16 -> 8 and 32 -> 16.
 *   sa_conv3d_pointwise_upcat: out = Wa . Ta(a) + up(p), a [B,Ca,D,H,W], p [B,Cout,Dp,Hp,Wp]
 *     upsampled with align_corners=True (Dp-1 <= (D-1)/2 per axis), weight [Ca][Cout],
 *     plus InstanceNorm partials as for sa_conv3d (parts = sa_conv3d_upcat_stat_parts(D, H, W)).
 *     Built for (8 -> 8, identity a) and (16 -> 16, transformed a). */
long sa_conv3d_upcat_stat_parts(int D, int H, int W);
int sa_conv3d_pointwise(const float *in, int B, int Cin, int D, int H, int W, const float *mean,
                        const float *rstd, int act, float slope, const float *gate_l,
                        const float *gate_r, const float *weight, int Cout, float *out, void *stream);
int sa_conv3d_pointwise_upcat(const float *a, int Ca, const float *a_mean, const float *a_rstd,
                              int a_act, const float *a_gl, const float *a_gr, const float *p,
                              int Dp, int Hp, int Wp, int B, int D, int H, int W, float slope,
                              const float *weight, int Cout, float *out, double *stats_partial,
                              void *stream);
/* sa_conv3d at stride 1 for Cin 8 -> Cout 8 or 2 (final_agg[1], final_agg[2], the classifier
 * pair), 16 -> 16 (down_layers[0][1], agg_layers[1][1..2]) and 32 -> 32 without gate
 * (down_layers[1][1], as two 16-channel halves per tile) with the D-taps as Winograd F(4,3) along
 * D: weight_wd [Cin][3 kh][3 kw][6][Cout] = G (points 0, +-1, +-2, inf) applied to the kernel's
 * D-taps (ops.conv3d_wd_weights).  The input's transform must include the InstanceNorm +
 * LeakyReLU (in_mean, act); statistics as for sa_conv3d with parts =
 * sa_conv3d_wd_stat_parts(Cout, D, H, W) (the 32-channel conv tiles like the 16-channel ones). */
long sa_conv3d_wd_stat_parts(int Cout, int D, int H, int W);
int sa_conv3d_wd(const float *in, int B, int Cin, int D, int H, int W, const float *weight_wd,
                 int Cout, const float *in_mean, const float *in_rstd, int act, float slope,
                 const float *gate_l, const float *gate_r, float *out, double *stats_partial,
                 void *stream);
/* sa_conv3d_wd's kernel variant (same products in the same order, bit-identical results):
 * 0 (default) wave-uniform scalar weights; 1 the per-channel weights staged in LDS with the input
 * slab, a channel ahead; 2 (8-input-channel convs) the two D-tiles' transform points paired in the
 * slab for packed FMAs; 3 variant 2 with the next channel's columns fetched by LDS-DMA.  For A/B
 * runs and tests. */
void sa_conv3d_wd_set_variant(int variant);
int sa_conv3d_wd_get_variant(void);
/* The stride-1 hourglass convs 8 -> 8 (final_agg[1..2]), 16 -> 16 (down_layers[0][1],
 * agg_layers[1][1..2]) and 32 -> 32 (down_layers[1][1]; hourglass.py:13-91, submodule.py:25-53)
 * as an implicit GEMM on
 * v_mfma_f32_16x16x32_f16 with split operands (csrc/conv3d_mfma.hip): same contract as
 * sa_conv3d_wd for an InstanceNorm + LeakyReLU producer without gate (in_mean / in_rstd per
 * (b, ci), required), fp32-level accuracy (hi/lo f16 activations, weights x 2^12 split the same
 * way; |w| < 8 required, which ops.py checks).
 *   sa_conv3d_mf_weights: [Cin][27][Cout] fp32 (ops.conv3d layout) -> the kernel's B-fragment
 *     table (sa_conv3d_mf_weights_size bytes, device memory; -1 for an unsupported shape).
 *     Cin = Cout = 8, 16 or 32.
 *   sa_conv3d_mf: out [B, Cout, D, H, W] raw conv of T(in) (pad 1, no bias) + InstanceNorm
 *     partials [B*Cout][parts][2], parts = sa_conv3d_mf_stat_parts(B, Cin, Cout, D, H, W);
 *     D*H*W < 2^30.
 *   sa_conv3d_mf_set_planes: output planes per block along D (0 = automatic; tests / A/B). */
long sa_conv3d_mf_weights_size(int Cin, int Cout);
int sa_conv3d_mf_weights(const float *weight, int Cin, int Cout, void *table, void *stream);
long sa_conv3d_mf_stat_parts(int B, int Cin, int Cout, int D, int H, int W);
int sa_conv3d_mf(const float *in, int B, int Cin, int D, int H, int W, const void *table, int Cout,
                 const float *in_mean, const float *in_rstd, float slope, float *out,
                 double *stats_partial, void *stream);
void sa_conv3d_mf_set_planes(int planes);
int sa_conv3d_mf_get_planes(void);
/* The hourglass's stride-2 16 -> 32 conv (down_layers[1][0], hourglass.py:27-33, submodule.py:25-53)
 * on the same split-f16 MFMA: in [B][16][D][H][W] with the producer's InstanceNorm (mean / rstd
 * [B*16]) + LeakyReLU(slope) and the optional feature-attention gate (sa_conv3d's gate_l / gate_r)
 * applied on load, out [B][32][Do][Ho][Wo] (Do = (D-1)/2+1, ...) and
 * optional float64 InstanceNorm partials [B*32][sa_conv3d_s2mf_stat_parts][2];
 * sa_conv3d_s2mf_weights turns the [16][27][32] kernel into its sa_conv3d_s2mf_weights_size-byte
 * table (|w| < 8).  Needs D*H*W < 2^30. */
long sa_conv3d_s2mf_weights_size(void);
int sa_conv3d_s2mf_weights(const float *weight, void *table, void *stream);
long sa_conv3d_s2mf_stat_parts(int Do, int Ho, int Wo);
int sa_conv3d_s2mf(const float *in, int B, int D, int H, int W, const void *table, const float *mean,
                   const float *rstd, float slope, const float *gate_l, const float *gate_r, float *out,
                   double *partial, void *stream);
/* The hourglass's two readers of the masked mono volume (down_layers[0][0], hourglass.py:27-33;
 * final_agg[0] over cat(orig, up(x)), hourglass.py:326-328) on the one-hot volume given by its
 * records (sa_mono_bin_records; rec_l [B,H,W] of the left pixels = the volume's W axis, rec_r
 * [B,H,D] of the right pixels = its D axis): each tap is one gather of W[bin][tap][:].
 *   sa_conv3d_onehot: as sa_conv3d on the volume [B, nbins, D, H, W] with the identity
 *     transform; built for nbins 8, stride 2, Cout 16; parts = sa_conv3d_onehot_stat_parts.
 *   sa_conv3d_pointwise_upcat_onehot: as sa_conv3d_pointwise_upcat with a = that volume
 *     (Ca = nbins = 8, Cout 8, identity transform); parts = sa_conv3d_upcat_stat_parts. */
long sa_conv3d_onehot_stat_parts(int Do, int Ho, int Wo);
int sa_conv3d_onehot(const float *rec_l, const float *rec_r, int B, int nbins, int D, int H, int W,
                     int stride, float gain, const float *weight, int Cout, float *out,
                     double *stats_partial, void *stream);
int sa_conv3d_pointwise_upcat_onehot(const float *rec_l, const float *rec_r, int nbins, float gain,
                                     const float *p, int Dp, int Hp, int Wp, int B, int D, int H,
                                     int W, const float *weight, int Cout, float *out,
                                     double *stats_partial, void *stream);
/* out = T(in) elementwise on a [B,C,D,H,W] volume (T as for sa_conv3d). */
int sa_vol_apply(const float *in, int B, int C, int D, int H, int W, const float *mean,
                 const float *rstd, int act, float slope, const float *gate_l, const float *gate_r,
                 float *out, void *stream);
/* mean/rstd of each of bc_count channels from the partials (count voxels each, biased
 * variance, rstd = 1/sqrt(var + eps)) — InstanceNorm3d statistics (affine=False). */
int sa_instnorm_finalize(const double *partial, int bc_count, long nparts, long count, float eps,
                         float *mean, float *rstd, void *stream);

/* convf1 + ReLU of the motion encoder (update.py:76, 85): direct KxK conv, Cin <= 8,
 * in [B,Cin,H,W] (batch stride in_bs) -> out [B,Cout,H,W] (batch stride out_bs). */
int sa_conv2d_small(const float *in, long in_bs, int B, int Cin, int H, int W, const float *weight,
                    const float *bias, int Cout, int ksize, int relu, float *out, long out_bs,
                    void *stream);

/* flow_head.conv2 (update.py:98-110): 3x3 / pad 1 conv, Cin (multiple of 8) -> Cout = 2,
 * weight in the module's [Cout][Cin][3][3] layout, bias may be NULL. */
int sa_conv2d_k3_narrow(const float *in, long in_bs, int B, int Cin, int H, int W, const float *weight,
                        const float *bias, int Cout, float *out, long out_bs, void *stream);

/* 3x3 / stride 1 / pad 1 conv (encoders extractor.py:6-300, update block update.py:46-110)
 * as fused Winograd F(2x2,3x3) on fp32 MFMA.  sa_conv2d_wino_weights transforms a
 * [Cout][Cin][3][3] kernel (Cin % 8 == 0) once into U, 16*Cin*Cout floats laid out
 * [16][Cin/8][4][Cout][2] (16-byte aligned); sa_conv2d_k3_wino:
 * in [N,Cin,H,W] (batch stride in_bs) -> out [N,Cout,H,W] (batch stride out_bs), + bias
 * (may be NULL), ReLU if relu != 0.  Needs Cin % 8 == 0 and Cout % 32 == 0. */
int sa_conv2d_wino_weights(const float *weight, int Cout, int Cin, float *U, void *stream);
int sa_conv2d_k3_wino(const float *in, long in_bs, int N, int Cin, int H, int W, const float *U,
                      int Cout, const float *bias, int relu, float *out, long out_bs, void *stream);
/* As sa_conv2d_k3_wino, plus the producer's epilogue applied while the input is loaded,
 * x -> act((x - m) * s + t) (m, s, t per channel with in_pstride 0 or per (image, channel)
 * with in_pstride Cin; NULL = 0 / 1 / 0; in_act 1 = ReLU; zero padding applies to the
 * result; Cin <= 512), and, if stats_partial != NULL, per-block float64 (sum, sum^2) of every
 * output channel, [N*Cout][parts][2] with parts = sa_conv2d_k3_wino_stat_parts(H, W), for
 * sa_instnorm_finalize. */
long sa_conv2d_k3_wino_stat_parts(int H, int W);
int sa_conv2d_k3_wino_ex(const float *in, long in_bs, int N, int Cin, int H, int W, const float *U,
                         int Cout, const float *bias, int relu, const float *in_m, const float *in_s,
                         const float *in_t, int in_pstride, int in_act, float *out, long out_bs,
                         double *stats_partial, void *stream);
/* Up to 8 independent sa_conv2d_k3_wino_ex convolutions in one launch (their blocks share
 * one grid, so a small conv's last, partly filled round of blocks is filled by the others).
 * All problems must have the same Cout % 64 == 0 outcome and either all or none carry an
 * input transform. */
typedef struct SaWinoProblem {
  const float *in;
  long in_bs;
  int N, Cin, H, W;
  const float *U;
  int Cout;
  const float *bias;
  int relu;
  const float *in_m, *in_s, *in_t;
  int in_pstride, in_act;
  float *out;
  long out_bs;
  double *stats_partial;
  /* row pitch (floats) of the input, output and gate planes when it differs from W (0 = W):
   * planes are [H][pitch] with columns W .. pitch - 1 zero in the input (they act as the right
   * zero padding) and kept zero in every output.  F(4x4) only (pitch % 4 == 0): a GRU level
   * whose width is not a multiple of 4 runs on it with its planes padded to a multiple of 4. */
  int pitch;
  /* residual epilogue (F(4x4) only; no statistics, no gate): out = oact(act(conv + bias) + skip'),
   * skip' = skip_act(skip * skip_s + skip_t) per output channel (NULL skip_s / skip_t = 1 / 0),
   * act = ReLU iff relu, skip_act / out_act 1 = ReLU; skip [N, Cout, H, pitch] with batch stride
   * skip_bs, 16-byte aligned.  skip = NULL: the plain epilogue.  (The closing
   * relu(relu(N2(c2)) + N3(skip)) of a BatchNorm residual block, extractor.py:41-60, with N2 folded
   * into the conv.) */
  const float *skip;
  long skip_bs;
  const float *skip_s, *skip_t;
  int skip_act, out_act;
} SaWinoProblem;
int sa_conv2d_k3_wino_multi(int nprob, const SaWinoProblem *probs, void *stream);

/* The same 3x3 convolutions as fused Winograd F(4x4,3x3) on fp32 MFMA (2.25 products per
 * output instead of 4).  sa_conv2d_wino4_weights transforms [Cout][Cin][3][3] (Cin % 8 == 0,
 * Cout % 32 == 0) once into U4, 36*Cin*Cout floats laid out [Cout/32][Cin/8][36][2][4][32]
 * (16-byte aligned).  sa_conv2d_k3_wino4_multi takes SaWinoProblem with U = U4 and needs
 * W % 4 == 0 and 16-byte aligned input planes (in, in_bs % 4 == 0); an input transform
 * (in_m / in_s / in_t / in_pstride, in_act 0 or 1 = ReLU, as sa_conv2d_k3_wino_ex) needs
 * Cin <= 256 (block_shape 0) or 512 (2) and no gate epilogue in the launch; bias, ReLU and the InstanceNorm partials
 * ([N*Cout][parts][2], parts = sa_conv2d_k3_wino4_stat_parts(H, W)) as sa_conv2d_k3_wino_ex. */
int sa_conv2d_wino4_weights(const float *weight, int Cout, int Cin, float *U4, void *stream);
/* U4 for the split block shape (block_shape 6 of sa_conv2d_k3_wino4_multi_gate: the Winograd-domain
 * products on f16 MFMA with hi/lo operand pairs): 36*Cin*Cout dwords in U4's layout, each dword
 * the f16 pair (hi, lo) of U * 2^12 (hi in the low half).  Needs |weight| < 16 (U * 2^12
 * within the f16 range). */
int sa_conv2d_wino4_weights_split(const float *weight, int Cout, int Cin, void *U4s, void *stream);
long sa_conv2d_k3_wino4_stat_parts(int H, int W);
int sa_conv2d_k3_wino4_multi(int nprob, const SaWinoProblem *probs, void *stream);
/* ConvGRU gates in the epilogue (update.py:16-27), per problem (gates[i].mode 0 = plain; gates
 * may be NULL).  v = conv + bias (no ReLU, no statistics), c = ctx plane of the same output
 * channel (ctx + co*H*W, batch stride ctx_bs), all planes 16-byte aligned:
 *   mode 1, conv over cat(h, x) with Cout = 2*Ch output channels (convz | convr):
 *           co < Ch: out[co] = sigmoid(v + c);  co >= Ch: out2[co - Ch] = sigmoid(v + c) * h[co - Ch]
 *   mode 2, conv over r*h (convq's r*h part): out[co] = (1 - z) h + z tanh((add + v) + c) with
 *           z, h, add (convq's x part) planes of channel co; out may be h itself (in place). */
typedef struct SaGateEpilogue {
  int mode;
  const float *ctx;
  long ctx_bs;
  const float *h;
  long h_bs;
  const float *z;
  long z_bs;
  const float *add;
  long add_bs;
  float *out2;
  long out2_bs;
  /* mode 3 (the flow head's two convs, update.py:98-110, of which the model reads output
   * channel 0 only, stereoanywhere.py:283): the conv (+ bias + ReLU) is conv1 over h08; head_w
   * = conv2's channel-0 filter [Cout][3][3] (Cout = the conv's output channels); each block
   * writes its channel block's partial conv2 sums over its tile plus a one-pixel border to
   * head_part (floats per image head_part_bs = sa_flow_head_part_size / N), and nothing to out;
   * sa_flow_head_reduce adds them up. */
  const float *head_w;
  float *head_part;
  long head_part_bs;
} SaGateEpilogue;
/* block_shape: 0 / 1 large blocks (8 waves, 64 Winograd tiles, one per CU), 2 small blocks (4
 * waves, 32 tiles, two per CU: shorter launches of few rounds fill the chip better), 6 split large
 * blocks (8 waves, 64 tiles x 32 output channels; every problem's U from
 * sa_conv2d_wino4_weights_split; the transformed inputs must stay below 65504 in magnitude, see the
 * guard of sa_conv2d_k3_wino4_launch).  Any other value is an error. */
int sa_conv2d_k3_wino4_multi_gate(int nprob, const SaWinoProblem *probs, const SaGateEpilogue *gates,
                                  int block_shape, void *stream);
/* sa_conv2d_k3_wino4_multi_gate with the split kernel's range guard (block_shape 6, guard != 0): a
 * block whose f16 operands overflowed (|transformed input| >= 65520, or an input not finite) writes
 * nothing and recomputes its work item right away on fp32 MFMA products (the split filters read as
 * hi + lo), so results never carry the overflow; every such block in parallel, no second launch.
 * sa_split_redo_blocks counts them.  Other block shapes ignore guard. */
int sa_conv2d_k3_wino4_launch(int nprob, const SaWinoProblem *probs, const SaGateEpilogue *gates,
                              int block_shape, int guard, void *stream);
/* Blocks of the split kernels (F(4x4) and sa_conv_direct_split) that the range
 * guards recomputed since the last reset (reset != 0 clears the count), -1 on error; synchronises the
 * device. */
long sa_split_redo_blocks(int reset);
/* 1x1 convolution (stride 1, no padding) as a GEMM on split-f16 MFMA (conv1x1.hip): the feature
 * encoder's output conv (extractor.py:149) and the mask head's 1x1 (update.py:159-162, 191).
 *   out[b][co][p] = scale * (bias[co] + sum_ci W[co][ci] x[b][ci][p]) over the flat H*W plane;
 *   each product as hi*hi + hi*lo + lo*hi of f16 pairs (22-bit operands), fp32 accumulation.
 * sa_conv1x1_weights: [Cout][Cin] fp32 -> the split weights (sa_conv1x1_weights_size(Cout, Cin)
 *   bytes, 16-byte aligned; |weight| < 16).
 * sa_conv1x1: x [B][Cin][H][W] (batch stride x_bs floats, 16-byte aligned, H*W % 4 == 0,
 *   Cin % 32 == 0), bias [Cout] or NULL, out [B][Cout][H][W] (batch stride out_bs).  A block whose
 *   inputs reach the f16 range (|x| >= 65504) recomputes its outputs with fp32 FMAs;
 *   sa_conv1x1_redo_blocks counts those blocks (reset != 0 clears; synchronises the device). */
long sa_conv1x1_weights_size(int Cout, int Cin);
int sa_conv1x1_weights(const float *weight, int Cout, int Cin, void *out, void *stream);
int sa_conv1x1(const float *x, long x_bs, int B, int Cin, int H, int W, const void *wsplit, int Cout,
               const float *bias, float scale, float *out, long out_bs, void *stream);
long sa_conv1x1_redo_blocks(int reset);
/* The tiled harness's data movement (mapreduce_v2/tile_wrapper.py:226-236, 169-185, 188-189;
 * tiler.hip):
 * sa_tile_gather_pad: src [C][H][W] (dense) -> out [ntiles][C][th + pt + pb][tw + pl + pr], tile t
 *   the rectangle at origin[2t] (row), origin[2t + 1] (column) (device int pairs), padded by edge
 *   replication (torch.cat of the tile views, then F.pad(..., mode="replicate")), bit-exact copies.
 * sa_tile_stitch: for every pixel of num / den [H][W], the ntiles entries tiles[3i .. 3i + 2] =
 *   (row, column, slot) in order (a rectangle listed twice adds twice), each covering it adds
 *   d * w to num and w to den, d = disp[slot * disp_ts + ty * dpitch + tx], w = wgt[ty * tw + tx];
 *   finalize != 0 then writes num = den > 0 ? num / max(den, 1e-4) : num (den untouched).  The
 *   reference's per-tile slice updates, per pixel in the same order: the same bits. */
int sa_tile_gather_pad(const float *src, int C, int H, int W, const int *origin, int ntiles, int th, int tw,
                       int pt, int pb, int pl, int pr, float *out, void *stream);
int sa_tile_stitch(const float *disp, long disp_ts, int dpitch, const int *tiles, int ntiles, int th, int tw,
                   const float *wgt, int H, int W, int finalize, float *num, float *den, void *stream);
/* The flow head fused (gate mode 3 above): floats of the partial-sum buffer of a conv over
 * [N, Cout, H, W] (-1 on bad shapes), and the reduction that finishes it: delta = bias0 + the
 * sum of the partials at each pixel (conv2's channel 0), then as sa_flow_update: coords_x +=
 * delta, flow_a / flow_b (optional, [N, 2, H, W]) = (coords_x - x, 0). */
long sa_flow_head_part_size(int N, int Cout, int H, int W);
int sa_flow_head_reduce(const float *part, int N, int Cout, int H, int W, const float *bias0, float *coords_x,
                        float *flow_a, long flow_a_bs, float *flow_b, long flow_b_bs, void *stream);

/* Direct KxK convolution (padding K/2, no bias) on fp32 MFMA for the encoder convs the
 * Winograd kernel does not cover (extractor.py:22-40, 91, 208):
 *   K = 7, S = 1, Cout % 64 == 0, Cin <= 4 (the 7x7 stems), and
 *   K = 3, S = 2, Cout 96 or a multiple of 128, Cin % 8 == 0, with the residual block's 1x1
 *   stride-2 downsample (weights wd, output out_ds) computed in the same launch.
 * sa_conv_direct_weights arranges a [Cout][Cin][K][K] kernel (K = 1 for the downsample, with
 * with_ds = 1 and the 3x3 conv's S) into sa_conv_direct_weights_size floats.  part / part_ds:
 * optional float64 InstanceNorm partials [N*Cout][sa_conv_direct_stat_parts(Ho, Wo)][2] for
 * sa_instnorm_finalize. */
long sa_conv_direct_weights_size(int Cout, int Cin, int K, int S, int with_ds);
int sa_conv_direct_weights(const float *weight, int Cout, int Cin, int K, int S, int with_ds, float *out,
                           void *stream);
long sa_conv_direct_stat_parts(int Ho, int Wo);
int sa_conv_direct(const float *in, long in_bs, int N, int Cin, int H, int W, int K, int S, const float *wg,
                   const float *wd, int Cout, float *out, long out_bs, float *out_ds, long out_ds_bs,
                   double *part, double *part_ds, void *stream);
/* The same convolutions with the products as exact f16 hi/lo pair products on MFMA (fp32
 * accumulation): wg / wd from sa_conv_direct_weights_split, which turns n arranged weights into
 * n dwords, the f16 pair (hi, lo) of w * 2^12 (needs |w| < 16). */
int sa_conv_direct_weights_split(const float *arranged, long n, void *out, void *stream);
int sa_conv_direct_split(const float *in, long in_bs, int N, int Cin, int H, int W, int K, int S, const void *wg,
                         const void *wd, int Cout, float *out, long out_bs, float *out_ds, long out_ds_bs,
                         double *part, double *part_ds, void *stream);
/* The stride-2 3x3 conv + fused 1x1 downsample of a residual block's output that was never
 * written (extractor.py:22-60: the feature encoder's stage boundary): the conv input is
 * relu(relu((c2 - mean) * rstd) + skip) per (image, channel) plane (mean / rstd [N*Cin], the
 * block's InstanceNorm of its conv2 output c2; skip the block input), formed while the patch is
 * staged with sa_norm_act's arithmetic, zero padding outside the image.  wg / wd as for
 * sa_conv_direct (split = 0) or sa_conv_direct_split (split = 1).  Replaces the block's closing
 * sa_norm_act pass.  sa_conv_direct_close_supported: 1 when a kernel exists (Cout = 96). */
int sa_conv_direct_close_supported(int K, int S, int Cout);
int sa_conv_direct_close(const float *c2, long c2_bs, const float *skip, long skip_bs, const float *mean,
                         const float *rstd, int N, int Cin, int H, int W, int K, int S, const void *wg,
                         const void *wd, int split, int Cout, float *out, long out_bs, float *out_ds,
                         long out_ds_bs, double *part, double *part_ds, void *stream);

/* Epilogues of the MIOpen 2-D convs (encoders extractor.py:6-300, update block update.py:64-110).
 * sa_plane_stats: InstanceNorm2d statistics (biased variance, eps) of each (b, c) plane of
 *   x [B,C,hw] (batch stride x_bs) -> mean, rstd [B*C].
 * sa_norm_act: out = act_out(act_in((x - m) * s + t) + skip_term), skip_term =
 *   act_skip((skip - skip_m) * skip_s + skip_t) (any of the three NULL = 0 / 1 / 0) or 0
 *   without skip;
 *   parameters per channel (pstride 0) or per (b, c) plane (pstride C); act 0 none,
 *   1 ReLU, 2 tanh; x, skip and out may be channel-slice views (batch strides); out may
 *   alias x. */
int sa_plane_stats(const float *x, long x_bs, int B, int C, long hw, float eps, float *mean,
                   float *rstd, void *stream);
int sa_norm_act(const float *x, long x_bs, int B, int C, long hw, const float *m, const float *s,
                const float *t, int pstride, int act_in, const float *skip, long skip_bs,
                const float *skip_m, const float *skip_s, const float *skip_t, int skip_pstride,
                int act_skip, int act_out, float *out, long out_bs, void *stream);

/* Live per-kernel timing for bench.py: when enabled, every launch of kernel `id`
 * is bracketed by hipEvents on the launch stream; sa_timing_read synchronises the
 * recorded events and returns their summed duration (ms) and count, then clears. */
enum {
  SA_K_CORR_PYRAMID = 0, SA_K_LOOKUP, SA_K_MONO_VOLUME, SA_K_SOFTARGMIN, SA_K_LSQ,
  SA_K_GRU_ZR, SA_K_GRU_OUT, SA_K_UPSAMPLE, SA_K_MISC, SA_K_CONV3D, SA_K_NORM, SA_K_CONV2D, SA_K_CONV_DIRECT,
  SA_K_CONV2D_W4, SA_K_SHEAR, SA_K_MONO_PYRAMID, SA_K_PLUMBING, SA_K_CONV_SMALL, SA_K_NARROW,
  SA_K_CONV1X1, SA_K_COUNT
};
/* Box-state probe (bench.py, outside timed regions; synchronises the device): `blocks` blocks of 4
 * waves run `iters` x 4 chained f16 MFMAs each; *mhz = the median over waves of the in-kernel shader
 * clock (delta s_memtime / delta s_memrealtime x 100 MHz), *ms = the kernel's event time. */
int sa_clock_probe(int blocks, int iters, double *mhz, double *ms);
int sa_timing_enable(int on);
int sa_timing_read(int kernel_id, double *total_ms, long *count);
const char *sa_kernel_name(int kernel_id);

#ifdef __cplusplus
}
#endif
#endif /* STEREOANYWHERE_HIP_H */
