/*
 * cgan3d — C-ABI of the MI355X (gfx950) HIP kernels behind the contrast-GAN-3D G+D train step.
 *
 * Drop-in boundary.  The reference (xqz-u/contrast-gan-3D) is pure Python over torch aten ops,
 * so there is no reference FFI; the entry points below replace the aten ops its hot path
 * dispatches and are bound from Python with ctypes by
 * contrast-gan-3d_amd/cgan3d_amd/_lib.py.  Each function cites the
 * reference call site whose arithmetic it implements.
 *
 * Conventions
 *  - Plain device pointers, sizes and a hipStream_t passed as void*; no torch types.
 *  - Activations are fp32 NDHWC (channels-last): element (n, d, h, w, c) at
 *    (((n*D + d)*H + h)*W + w)*C + c.  For C == 1 this equals the reference's NCDHW layout,
 *    so the generator input/output and the critic input cross the boundary without copies.
 *  - Weights stay in torch layout ([Cout, Cin, k, k, k] for Conv3d, [Cin, Cout, k, k, k] for
 *    ConvTranspose3d); the geometry carries the strides of the two channel indices.
 *  - The library never allocates: scratch comes from caller-provided workspace.
 *  - All launches are asynchronous on `stream`; no host synchronisation; every entry point is
 *    safe to capture in a hipGraph.
 *  - Return 0 on success; otherwise an errno-style code and cgan3d_get_last_error() (per host
 *    thread) describes the failure.  Shapes are validated on the host before any launch.
 */
#ifndef CGAN3D_H_
#define CGAN3D_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CGAN3D_OK 0
#define CGAN3D_EINVAL 22
#define CGAN3D_EHIP 100

/* Conv geometry.  "Gathered" operand G has spatial dims (di,hi,wi) and `cin` channels; the
 * voxel-aligned operand/output O has dims (do_,ho,wo) and `cout` channels.  Tap t = (td,th,tw)
 * of a k^3 kernel links O-voxel o and G-voxel i by
 *   transposed == 0 :  i = o*stride - pad + t   (Conv3d forward; ConvTranspose3d input-grad)
 *   transposed == 1 :  o = i*stride - pad + t   (ConvTranspose3d forward; Conv3d input-grad)
 * reflect != 0 (transposed == 0 only) mirrors out-of-range i (torch padding_mode="reflect"),
 * otherwise out-of-range taps contribute zero.  Weight element for (G channel a, O channel b,
 * tap index t = (td*k + th)*k + tw) is w[a*w_sa + b*w_sb + t]. */
typedef struct cgan3d_conv_geom {
  int32_t n;
  int32_t di, hi, wi;
  int32_t do_, ho, wo;
  int32_t cin, cout;
  int32_t k, stride, pad;
  int32_t transposed;
  int32_t reflect;
  int64_t w_sa, w_sb;
  int32_t w_packed;  /* 1: w is cgan3d_pack_weights() output [tap][a][b] f32, b contiguous;
                      * 2: halo format, bf16 [tap][b][a] with 16-byte granules of a XOR-swizzled
                      *    by (b mod a/8) — prec BF16, cin 32|64, cout%16==0, no reflect, k<=4,
                      *    stride<=2 (cgan3d_halo_eligible);
                      * 3: small-grid K-split format, bf16 [b][tap][a] — prec BF16, k 4, cin%8==0,
                      *    cout%8==0 (the critic's middle layers; cgan3d_packed_format) */
  int32_t prec;      /* CGAN3D_PREC_F32 (exact f32 MFMA) or CGAN3D_PREC_BF16 (bf16 MFMA, f32 accumulate) */
  int32_t planar;    /* 1: a 2-D convolution (nn.Conv2d / nn.ConvTranspose2d of the is_2D variants,
                      * model/blocks.py:22-27, experiments/conf_2D.py): di == do_ == 1, the depth
                      * axis is a pass-through (kernel 1, stride 1, pad 0, one parity class), the
                      * kernel has k*k taps t = th*k + tw and weights are [Cout, Cin, k, k] /
                      * [Cin, Cout, k, k].  Runs on the generic f32 paths (implicit GEMM for
                      * cout >= 2, any cout; the VALU cout == 1 kernels), w_packed 0 or 1 */
} cgan3d_conv_geom;

#define CGAN3D_PREC_F32 0
#define CGAN3D_PREC_BF16 1

#define CGAN3D_ACT_NONE 0
#define CGAN3D_ACT_RELU 1
#define CGAN3D_ACT_LRELU 2
#define CGAN3D_ACT_TANH 3
/* epilogue of the critic's first-layer input-grad only (cgan3d_conv3d_neg_dtanh_ok): the generator's
 * adversarial gradient taken through its output tanh and added to the loss part in place,
 *   out = residual - v * (1 - mask_src^2)     (mask_src = the generator's tanh output att,
 * opt_hat = subopt - att: generator.py:86-88; Trainer.py:148-157), so the generator's losses and
 * their gradient can be computed beside the critic update and only this fold stays on the path. */
#define CGAN3D_ACT_NEG_DTANH 4

/* Fused epilogue: v = acc (+ bias[c]); v = act(v); v *= (mask_src > 0 ? 1 : slope) if mask_src;
 * v += residual if residual; out = v; if out2: out2 = minuend - v (cout == 1 only).
 * stats != NULL: per-block BatchNorm partials (sum, M2, count) of v, consumed by
 * cgan3d_bn_finalize; size cgan3d_conv3d_stats_floats().
 * Fused BatchNorm statistics (forward and input-grad kernels of the k7 / halo / implicit-GEMM
 * paths, and cgan3d_reflect_fold_ex): each block b of the launch writes its per-channel partial
 * pair into a channel-major slab bn_part[(q * cout + c) * bn_slots + b] (q = 0, 1; no atomics),
 * bn_slots = cgan3d_conv3d_bn_slots() / cgan3d_reflect_fold_slots():
 *  bn_mode 1: v is the BatchNorm input z: rows sum v (c), M2 of v about the block mean (cout + c)
 *             and the block's voxel count (row 2*cout): (2*cout + 1) * bn_slots floats
 *             (cgan3d_bn_finalize_slab, Chan's combine);
 *  bn_mode 2: v is dL/dy of a BatchNorm layer y = act(z * scale + shift) whose input z has the
 *             layout of this output: (sum g, sum g*xhat) with g = v * act'(z*scale + shift),
 *             xhat = (z - mean) * invstd (cgan3d_bn_backward_finalize_slab). */
/* BatchNorm statistics into fp64 accumulators instead of a slab (bf16 generator path): every block
 * of the producing launch adds its per-channel pair into acc_out[(r * 2 + q) * cout + c] (replica
 * r = block % reps; reps * 2 * cout doubles, zero before the launch), consumed by
 * cgan3d_bn_apply_acc / cgan3d_bn_backward_acc / cgan3d_bn_backward_acc_fold (finalize folded into
 * the elementwise launch: one launch per BatchNorm layer and direction, model/blocks.py:50-53):
 *   acc_mode 3 (forward): q = 0 sum v, q = 1 sum v^2 (v = the BatchNorm input z, this output);
 *   acc_mode 4 (input-grad): the pair of bn_mode 2 — sum g, sum g*xhat — with bn_z / bn_ss / bn_mi /
 *              bn_act of the epilogue (and bn_fold on the k7 input-grad).
 * Producers (cgan3d_bn_fuse_ok): the halo-tiled kernels (w_packed 2, incl. the stride-2 16 <-> 32
 * ones) and the generator's 1 -> 16 k7 MFMA kernel (first conv forward, last conv input-grad). */
typedef struct cgan3d_bn_fuse {
  double* acc_out;
  int32_t acc_mode;     /* 3 or 4 */
  int32_t reps;         /* replicas of acc_out (1..64) */
} cgan3d_bn_fuse;

/* BatchNorm of the conv's INPUT, applied by the ResNet-block kernel while it stages its halo (round 5:
 * the chain's elementwise BatchNorm launches folded into the next conv; model/blocks.py:56-88).  The
 * launch's x_bf16 is then the raw tensor of the previous BatchNorm layer and every block finalizes
 * that layer's statistics from the fp64 replicas itself:
 *   mode 1 (forward, cgan3d_bn_apply_acc without a residual): x_bf16 = the bf16 z, acc = its (sum,
 *          sum of squares) replicas; the conv input is act(z * scale + shift); one block writes
 *          scale_shift / mean_invstd / the running buffers / num_batches_tracked;
 *   mode 2 (input-grad, cgan3d_bn_backward_acc): x_bf16 = the bf16 dL/dy of the layer, z its bf16
 *          BatchNorm input, acc its (sum g, sum g * xhat) replicas, scale_shift / mean_invstd those of
 *          its forward; the conv input is dL/dz; one block writes dgamma / dbeta (added when
 *          accumulate).
 * out_bf16 receives the applied input at every voxel (bf16, same layout): the operand the layer's
 * weight gradient reads.  zero / zero_n: doubles zeroed by the launch (an accumulator the stream is
 * done with, as cgan3d_bn_apply_acc).  Only launches with cgan3d_conv3d_bn_pre_ok take it. */
typedef struct cgan3d_bn_pre {
  int32_t mode;
  const void* z;                /* mode 2 */
  const double* acc;
  int32_t reps;                 /* 1..64 */
  int64_t nvox;
  const float* gamma;
  const float* beta;            /* mode 1 */
  float* running_mean;          /* mode 1, optional */
  float* running_var;           /* mode 1, optional */
  int64_t* num_batches_tracked; /* mode 1, optional */
  float momentum;
  float eps;
  float* scale_shift;           /* mode 1: written; mode 2: read */
  float* mean_invstd;           /* mode 1: written; mode 2: read */
  float* dgamma;                /* mode 2, optional */
  float* dbeta;                 /* mode 2, optional */
  int32_t accumulate;
  int32_t act;
  float slope;
  void* out_bf16;
  double* zero;
  int32_t zero_n;
} cgan3d_bn_pre;

typedef struct cgan3d_epilogue {
  const float* bias;
  const float* residual;
  const float* mask_src;
  const float* minuend;
  float* out2;
  float* stats;
  int32_t act;
  float slope;
  float* bn_part;
  int32_t bn_mode;             /* 0 off, 1 forward statistics, 2 backward statistics */
  int32_t bn_slots;            /* slot stride of bn_part (must equal the launch's slot count) */
  const float* bn_z;           /* mode 2: the BatchNorm input z */
  const float* bn_ss;          /* mode 2: [scale | shift] */
  const float* bn_mi;          /* mode 2: [mean | invstd] */
  int32_t bn_act;              /* mode 2: the activation after the BatchNorm */
  float bn_slope;
  const void* x_bf16;          /* optional bf16 copy of the input x (same layout): the ResNet-block
                                * kernel stages its halo from it (half the bytes, no conversion) */
  int32_t bn_fold;             /* mode 2 on the padded output grid of a k7 input-grad (the last
                                * conv's, generator.py:78-84): the statistics are those of the
                                * reflect-folded tensor (pad bn_fold), bn_z lives on the unpadded
                                * grid; see cgan3d_bn_backward_slab_fold.  0 otherwise. */
  const cgan3d_bn_fuse* fuse;  /* NULL, or the statistics into fp64 accumulators (above) */
  int32_t out_bf16;            /* bit 0 (1): the output y and bn_z are bf16 arrays (same layout, passed
                                * through the float* / const float* slots); bit 1 (2): the residual is
                                * bf16 (the ResNet-block kernel only): the generator's BatchNorm inputs
                                * and their gradients kept in bf16 (round 4) — only launches with
                                * cgan3d_conv3d_out_bf16_ok accept it, every other launch rejects it */
  const cgan3d_bn_pre* pre;    /* NULL, or the input's BatchNorm applied while staging (above) */
} cgan3d_epilogue;

/* 1 when the launch of g can take cgan3d_epilogue.pre (the ResNet-block kernel: mode 1 on the forward
 * geometry, mode 2 on the input-grad one). */
int32_t cgan3d_conv3d_bn_pre_ok(const cgan3d_conv_geom* g);

/* 1 when the forward-style launch of g honours cgan3d_epilogue.out_bf16: the 1 -> 16 k7 MFMA kernel
 * (first conv forward; last conv input-grad, its folded statistics reading a bf16 z), the S2T
 * kernel (ConvTranspose3d 32 -> 16 forward; the first downsampling conv's input-grad with acc_mode 4
 * statistics reading a bf16 z), the ResNet-block kernel (Conv3d 64 -> 64 k3 forward / input-grad
 * with the bf16 input shadow; bit 1 there: a bf16 skip gradient as the residual) and the 64 -> 32
 * stride-2 transposed kernel (ConvTranspose3d 64 -> 32 forward, the second downsampling conv's
 * input-grad; round 5). */
int32_t cgan3d_conv3d_out_bf16_ok(const cgan3d_conv_geom* g);

/* 1 when the geometry's launch can produce cgan3d_bn_fuse accumulators. */
int32_t cgan3d_bn_fuse_ok(const cgan3d_conv_geom* g);
/* 1 when the input-grad geometry takes the CGAN3D_ACT_NEG_DTANH epilogue (the critic's first layer,
 * discriminator.py:55-60, 1 -> 8 k4 s2 p1). */
int32_t cgan3d_conv3d_neg_dtanh_ok(const cgan3d_conv_geom* g);
/* 1 when the launch of g goes to the direct cin == 1 stride-1 transposed kernel (the critic's
 * last-layer input-grad, exact fp32): it reads torch-layout weights (w_packed 0), no packed copy. */
int32_t cgan3d_conv3d_cin1t(const cgan3d_conv_geom* g);
/* Blocks of the input-grad launch when the geometry (the critic's first layer) can write the
 * per-block sum of squares of its output: then cgan3d_epilogue.stats = float[blocks], the blocks
 * of sample s being [s * blocks / n, (s + 1) * blocks / n); 0 when it cannot. */
int64_t cgan3d_conv3d_sumsq_blocks(const cgan3d_conv_geom* g);

const char* cgan3d_version(void);
const char* cgan3d_get_last_error(void);
/* Launch-shape / kernel choice (process-wide; set before building plans).  Seven keys, every value a
 * correct configuration (anything else: CGAN3D_EINVAL): 9 voxel chunks of the ResNet weight grad
 * (default 28, 0 = generic kernel); 10 blocks of the stride-2 weight grads (default 128 for the 16 <-> 32
 * level, half of it for the 32 <-> 64 level; 0 = generic);
 * 13 output planes per streamed last-conv block (0 auto, 8, 16, -1 = Toeplitz kernel); 15 ResNet convs
 * on conv_k3m and the 32 <-> 64 stride-2 pair on conv_t64 / conv_f64 (1, default) or all of them on the
 * round-3 halo kernels conv_k3 / conv_halo (0); 16 ResNet weight grads on wgrad_k3m (1, default) or
 * wgrad_k3 (0); 20 most blocks of a k7 weight grad (default 512); 21 (round 6) output planes per
 * streamed-plane 1 <-> 16 k7 block (0 auto, 1..64; -1 = the k7m_n2w / k7m_wg kernels). */
int cgan3d_set_tuning(int32_t key, int32_t value);

/* --- convolutions (model/blocks.py:29-38 Conv3d / ConvTranspose3d; generator.py:78-84 last
 *     conv; discriminator.py:24-80 critic convs; and their autograd backward) --- */
int64_t cgan3d_conv3d_stats_floats(const cgan3d_conv_geom* g);
/* Re-layout a torch-layout weight (strides w_sa, w_sb of g) into the packed [tap][a][b] rows the
 * forward/input-grad kernels read as contiguous vectors (once per optimiser step). */
int64_t cgan3d_packed_weight_floats(const cgan3d_conv_geom* g);
/* 1 when the geometry (ignoring w_packed) can run the halo-tiled bf16 kernel (w_packed = 2). */
int32_t cgan3d_halo_eligible(const cgan3d_conv_geom* g);
/* The packed weight format the fastest kernel for this geometry reads (3, 2 or 1; see w_packed). */
int32_t cgan3d_packed_format(const cgan3d_conv_geom* g);
int cgan3d_pack_weights(const cgan3d_conv_geom* g, const float* w, float* wp, void* stream);
/* Many packs in one launch: `descs` is a DEVICE array of n descriptors (built once; the pointers
 * are stable), `max_total` the largest element count (taps*cin*ldb or taps*cin*cout) among them. */
typedef struct cgan3d_pack_desc {
  const float* w;
  float* wp;
  int64_t sa, sb;
  int32_t taps, cin, cout, ldb;
  int32_t format;  /* w_packed value: 1 f32 [tap][a][b] (ldb-padded), 2 halo bf16 [tap][b][a],
                    * 3 K-split bf16 [b][tap][a] */
  int32_t reserved;
} cgan3d_pack_desc;
int cgan3d_pack_weights_multi(const cgan3d_pack_desc* descs, int32_t n, int64_t max_total, void* stream);
/* One optimiser step in one launch (optimizer.step(), Trainer.py:135,158): cgan3d_adam_tick +
 * cgan3d_adam over the arena + cgan3d_pack_weights_multi over `descs` (ndesc may be 0), same bits:
 * each updated parameter is also written into every packed copy whose source weight holds it
 * (descriptor weights must be contiguous views into `param`).  `ticket`: two uint32 words, zeroed
 * once by the caller and left zeroed (the last block out advances the step counter). */
/* Adam over a part of an arena ahead of the rest, with the step the coming cgan3d_adam_pack of the
 * remainder will advance to (step + 1) and without advancing it: the generator's layers whose
 * gradients are complete early in the backward are updated beside its tail. */
int cgan3d_adam_range(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                      const float* hyper, void* stream);
int cgan3d_adam_pack(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float* hyper,
                     const cgan3d_pack_desc* descs, int32_t ndesc, uint32_t* ticket, void* stream);
int cgan3d_conv3d_fwd(const cgan3d_conv_geom* g, const float* x, const float* w, float* y,
                      const cgan3d_epilogue* ep, void* stream);
/* weight gradient: dw[a*w_sa + b*w_sb + t] (+)= sum_o G_gathered(o,t,a) * O(o,b) with the
 * transposed==0 mapping.  Workspace: cgan3d_conv3d_wgrad_ws_floats() floats. */
int64_t cgan3d_conv3d_wgrad_ws_floats(const cgan3d_conv_geom* g);
int cgan3d_conv3d_wgrad(const cgan3d_conv_geom* g, const float* gathered, const float* aligned,
                        float* dw, int32_t accumulate, float* ws, void* stream);
/* The same with optional bf16 shadows of both operands (same layouts, NULL = none): the ResNet-
 * block weight-grad kernel then stages them as they are (bit-identical: it rounds to bf16 anyway). */
/* `accumulate` of the weight-gradient entry points is a flag word: CGAN3D_WGRAD_ACCUMULATE adds
 * into dw instead of overwriting it (a caller that zeroes a whole gradient arena once per update
 * passes it for every layer, so no per-layer memset of dw is issued); CGAN3D_WGRAD_WS_CLEAN promises
 * that ws is all-zero on entry and asks that the kernels that sum into ws by atomics leave it
 * all-zero again (no per-layer memset of ws; the workspace must then be used by clean calls only). */
#define CGAN3D_WGRAD_ACCUMULATE 1
#define CGAN3D_WGRAD_WS_CLEAN 2
/* with CGAN3D_WGRAD_WS_CLEAN on an atomic-workspace geometry: leave the result in the packed
 * workspace ([tap][a][b]); the caller later moves it into dw, and re-zeroes the workspace, with
 * cgan3d_wgrad_unpack_multi — one launch for a whole network's weight gradients */
#define CGAN3D_WGRAD_DEFER_UNPACK 4
typedef struct cgan3d_unpack_desc {
  float* ws;     /* packed [tap][a][b] workspace of one deferred weight gradient (left zeroed) */
  float* dw;     /* dw[a*sa + b*sb + tap] (+)= ws[(tap*cin + a)*cout + b] */
  int64_t sa, sb;
  int32_t taps, cin, cout, accumulate;
} cgan3d_unpack_desc;
/* `descs`: a DEVICE array of n descriptors; max_total = the largest taps*cin*cout among them */
int cgan3d_wgrad_unpack_multi(const cgan3d_unpack_desc* descs, int32_t n, int64_t max_total, void* stream);
/* on a geometry whose weight gradient reduces per-block partials (cgan3d_conv3d_wgrad_partials > 0:
 * the ResNet-block k3 kernel): leave the partials in ws and skip the reduce; the caller sums them into
 * dw later with cgan3d_wgrad_reduce_multi — one launch for every ResNet layer of a backward (round 5) */
#define CGAN3D_WGRAD_DEFER_REDUCE 8
/* partial sums the weight gradient of g leaves in ws (ws[p][27][cout][cin], p < P), 0 if it sums
 * another way */
int32_t cgan3d_conv3d_wgrad_partials(const cgan3d_conv_geom* g);
typedef struct cgan3d_reduce_desc {
  const float* ws;  /* P partials [p][27][cout][cin] of one deferred weight gradient */
  float* dw;        /* dw[a*sa + b*sb + tap] (+)= sum_p ws[p][tap][b][a] */
  int64_t sa, sb;
  int32_t P, cin, cout, accumulate;
} cgan3d_reduce_desc;
/* 1 <= n <= 16 descriptors (passed by value into the launch) */
int cgan3d_wgrad_reduce_multi(const cgan3d_reduce_desc* descs, int32_t n, void* stream);
/* 1 if the weight gradient of `g` sums into its workspace by atomics (the geometries that may take
 * CGAN3D_WGRAD_WS_CLEAN), 0 if not, -1 on an invalid geometry.  Round 6: the bf16 geometries (cout 4-64) return 0 —
 * their weight gradients write per-block partials into ws and sum them into dw in a fixed order (the
 * k7 and critic first-layer kernels' partial rows, the generic bf16 kernel's partial slabs, the ResNet /
 * stride-2 kernels' partials), so the bf16 step's gradients do not depend on the order blocks finish;
 * the exact-f32 generic kernels keep their atomic workspaces. */
int cgan3d_conv3d_wgrad_ws_mode(const cgan3d_conv_geom* g);
/* 1 when the kernel this geometry dispatches to reads ONLY the bf16 shadows of its operands once
 * they are given, so the caller may leave their fp32 tensors unwritten: role 0 = cgan3d_conv3d_fwd
 * with cgan3d_epilogue.x_bf16 (the stride-2 16 <-> 32 kernels, the 16 -> 1 k7 conv, the ResNet-block
 * convs), role 1 = cgan3d_conv3d_wgrad_ex
 * with both shadows (ResNet / stride-2 kernels) or, for a k7 conv with a single-channel side, the
 * multi-channel operand's shadow (the bf16 MFMA kernel).  0 otherwise. */
int32_t cgan3d_conv3d_shadow_only(const cgan3d_conv_geom* g, int32_t role);
/* 1 when the geometry's launch accepts cgan3d_epilogue.bn_fold (the bf16 k7 input-grad kernel). */
int32_t cgan3d_conv3d_bn_fold_ok(const cgan3d_conv_geom* g);
int cgan3d_conv3d_wgrad_ex(const cgan3d_conv_geom* g, const float* gathered, const float* aligned,
                           float* dw, int32_t accumulate, float* ws, const void* gathered_bf16,
                           const void* aligned_bf16, void* stream);

/* Several independent weight gradients in ONE launch (the critic's middle layers once the penalty's
 * forward-mode chain is done, discriminator.py:42-68: grids of 100-300 blocks that each leave most of
 * the chip idle and pay a launch apiece): item i adds sum_o G_i(o*s - p + t, a) O_i(o, b) into its
 * packed [t][a][b] workspace ws[i], all-zero on entry, exactly as cgan3d_conv3d_wgrad_ex with
 * CGAN3D_WGRAD_ACCUMULATE | CGAN3D_WGRAD_WS_CLEAN | CGAN3D_WGRAD_DEFER_UNPACK would (then
 * cgan3d_wgrad_unpack_multi).  1 <= n <= 4; every geometry cgan3d_conv3d_wgrad_group_ok. */
int32_t cgan3d_conv3d_wgrad_group_ok(const cgan3d_conv_geom* g);

/* The critic's k4 s2 p1 middle-layer weight gradients (discriminator.py:42-68, their penalty update,
 * Trainer.py:108-142) from a staged input window per output tile (every tap a row shift inside it),
 * bf16 MFMA, fp32 accumulation (round 5, csrc/wgrad_sk.hip): per-block partial tiles into ws[i]
 * (cgan3d_conv3d_wgrad_sk_ws_floats(g) floats, any contents), then one reduce launch that ADDS the
 * sums into dw[i] (torch layout, g.w_sa / g.w_sb).  1 <= n <= 4; geometries cgan3d_conv3d_wgrad_sk_ok:
 * bf16, not transposed, (cin, cout) = (8, 16) / (16, 32) / (32, 64), input = 2 x output, output
 * divisible by the variant's tile (d x h x w: 4 x 8 x 16 for 8 -> 16, 4 x 4 x 8 for 16 -> 32, 4 x 4 x 4 for
 * 32 -> 64).  Two launches. */
int32_t cgan3d_conv3d_wgrad_sk_ok(const cgan3d_conv_geom* g);
int64_t cgan3d_conv3d_wgrad_sk_ws_floats(const cgan3d_conv_geom* g);
int cgan3d_conv3d_wgrad_sk(const cgan3d_conv_geom* geoms, const float* const* gathered, const float* const* aligned,
                           float* const* ws, float* const* dw, int32_t n, void* stream);
int cgan3d_conv3d_wgrad_group(const cgan3d_conv_geom* geoms, const float* const* gathered,
                              const float* const* aligned, float* const* ws, int32_t n, void* stream);

/* --- BatchNorm3d, training mode (model/blocks.py:26-27,45; torch.nn.BatchNorm3d) --- */
int cgan3d_bn_finalize(const float* stats, int64_t nblk, int32_t c, const float* gamma,
                       const float* beta, float* running_mean, float* running_var,
                       int64_t* num_batches_tracked, float momentum, float eps,
                       float* scale_shift, float* mean_invstd, void* stream);
/* y_bf16 (optional, NULL = none): a bf16 copy of y written by the same pass (the input of the
 * next ResNet-block conv, cgan3d_epilogue.x_bf16).  y may be NULL when y_bf16 is given (every
 * reader of the output takes the bf16 copy); the same holds for cgan3d_bn_apply_slab. */
int cgan3d_bn_apply(const float* z, int64_t nvox, int32_t c, const float* scale_shift,
                    int32_t act, float slope, const float* residual, float* y, void* y_bf16, void* stream);
/* Slots of a launch's fused BatchNorm slab (cgan3d_epilogue bn_part); 0 when the geometry's
 * kernel has no fused statistics. */
int64_t cgan3d_conv3d_bn_slots(const cgan3d_conv_geom* g);
/* Forward statistics from a bn_mode-1 slab of nslots slots over nvox voxels (fp64 Chan combine):
 * scale_shift, mean_invstd and the running statistics (biased variance to normalise, unbiased
 * into running_var, torch momentum), for cgan3d_bn_apply. */
int cgan3d_bn_finalize_slab(const float* part, int32_t nslots, int32_t c, int64_t nvox, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            int64_t* num_batches_tracked, float momentum, float eps, float* scale_shift,
                            float* mean_invstd, void* stream);
/* Backward from a bn_mode-2 slab (filled by the kernel that produced dy): dgamma = sum g*xhat,
 * dbeta = sum g (+= when accumulate), then dz = gamma*invstd*(g - mean g - xhat*mean(g*xhat)).
 * ws: 3*c floats. */
/* cgan3d_bn_finalize_slab followed by cgan3d_bn_apply, as ONE launch when the slab is small
 * (every block combines the statistics itself; block 0 writes scale_shift / mean_invstd and the
 * running buffers) — blocks.py:26-27,45 BatchNorm3d train forward + activation (+ residual). */
int cgan3d_bn_apply_slab(const float* part, int32_t nslots, int32_t c, int64_t nvox, const float* gamma,
                         const float* beta, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                         float momentum, float eps, float* scale_shift, float* mean_invstd, const float* z,
                         int32_t act, float slope, const float* residual, float* y, void* y_bf16,
                         void* stream);
/* dz_bf16 (optional): bf16 copy of dz, as y_bf16 above (input of a ResNet-block input-grad);
 * dz may then be NULL. */
int cgan3d_bn_backward_slab(const float* dy, const float* z, int64_t nvox, int32_t c, const float* part,
                            int32_t nslots, const float* scale_shift, const float* mean_invstd,
                            const float* gamma, int32_t act, float slope, float* dgamma, float* dbeta,
                            float* dz, int32_t accumulate, float* ws, void* dz_bf16, void* stream);
int64_t cgan3d_bn_backward_ws_floats(int64_t nvox, int32_t c);
/* cgan3d_bn_backward_slab whose dy is the reflect fold (pad `pad`, torch "reflect") of `padded`
 * ([n][d+2pad][h+2pad][w+2pad][c]), folded on the fly — the input-grad of the generator's last conv
 * (generator.py:78-84) without materialising dy; the slab comes from that conv's launch with
 * cgan3d_epilogue.bn_fold = pad.  dz may be NULL when dz_bf16 is given. */
int cgan3d_bn_backward_slab_fold(const float* padded, const float* z, int32_t n, int32_t d, int32_t h, int32_t w,
                                 int32_t c, int32_t pad, const float* part, int32_t nslots, const float* scale_shift,
                                 const float* mean_invstd, const float* gamma, int32_t act, float slope,
                                 float* dgamma, float* dbeta, float* dz, int32_t accumulate, float* ws,
                                 void* dz_bf16, void* stream);
/* The same two passes from fp64 accumulators (cgan3d_bn_fuse acc_mode 3 / 4 of the producing conv:
 * acc[r][2][c], r < reps) instead of a slab, finalize folded into the elementwise launch (every
 * block combines the replicas itself; block 0 publishes scale_shift / mean_invstd / the running
 * buffers, or dgamma / dbeta): one launch per BatchNorm layer and direction.  Block 0 also zeroes
 * `zero_n` doubles at `zero` (an accumulator the stream is done with; NULL / 0: none).
 * blocks.py:26-27,45 BatchNorm3d train forward + act (+ residual), and its autograd backward. */
/* in_bf16 (round 4): 1 when z (apply) / dy and z (backward) / padded and z (fold) are bf16 arrays
 * (the conv that produced them had cgan3d_epilogue.out_bf16); the statistics still come from the
 * producer's fp32 values through the accumulators. */
int cgan3d_bn_apply_acc(const double* acc, int32_t reps, int32_t c, int64_t nvox, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                        float momentum, float eps, float* scale_shift, float* mean_invstd, const void* z,
                        int32_t act, float slope, const float* residual, float* y, void* y_bf16, double* zero,
                        int32_t zero_n, int32_t in_bf16, void* stream);
int cgan3d_bn_backward_acc(const void* dy, const void* z, int64_t nvox, int32_t c, const double* acc,
                           int32_t reps, const float* scale_shift, const float* mean_invstd, const float* gamma,
                           int32_t act, float slope, float* dgamma, float* dbeta, float* dz, int32_t accumulate,
                           void* dz_bf16, double* zero, int32_t zero_n, int32_t in_bf16, void* stream);
/* cgan3d_bn_backward_slab_fold with the statistics from accumulators (the last conv's input-grad
 * launch with cgan3d_bn_fuse acc_mode 4 and bn_fold), one launch. */
int cgan3d_bn_backward_acc_fold(const void* padded, const void* z, int32_t n, int32_t d, int32_t h, int32_t w,
                                int32_t c, int32_t pad, const double* acc, int32_t reps, const float* scale_shift,
                                const float* mean_invstd, const float* gamma, int32_t act, float slope,
                                float* dgamma, float* dbeta, float* dz, int32_t accumulate, void* dz_bf16,
                                double* zero, int32_t zero_n, int32_t in_bf16, void* stream);

/* accumulate != 0: dgamma/dbeta += this batch's gradients (a module called on several batches in
 * one step, e.g. the BatchNorm critic on the real and the fake batch, Trainer.py:119-121). */
int cgan3d_bn_backward(const float* dy, const float* z, int64_t nvox, int32_t c,
                       const float* scale_shift, const float* mean_invstd, const float* gamma,
                       int32_t act, float slope, float* dgamma, float* dbeta, float* dz,
                       int32_t accumulate, float* ws, void* stream);

/* --- reductions / elementwise --- */
/* Several channel sums in two launches (the critic's bias gradients, Trainer.py:133 backward of
 * model/discriminator.py's conv biases): `descs` is a DEVICE array of n descriptors (stable
 * pointers, built once), each summing x[nvox][c] per channel into out[c] (+= when accumulate)
 * through its own workspace of nblk * c doubles; c must divide 256 and be <= cmax.  Sums in fp64. */
typedef struct cgan3d_csum_desc {
  const float* x;
  float* out;
  double* ws;
  int64_t nvox;
  int32_t c;
  int32_t accumulate;
} cgan3d_csum_desc;
int cgan3d_channel_sum_multi(const cgan3d_csum_desc* descs, int32_t n, int32_t nblk, int32_t cmax, void* stream);
int64_t cgan3d_channel_sum_ws_floats(int64_t nvox, int32_t c);
int cgan3d_channel_sum(const float* x, int64_t nvox, int32_t c, float* out, float* ws,
                       void* stream);
int cgan3d_reflect_fold(const float* padded, float* out, int32_t n, int32_t d, int32_t h,
                        int32_t w, int32_t c, int32_t pad, void* stream);
/* reflect_fold(_ex) for the 2-D variants (nn.Conv2d padding_mode="reflect", generator.py:19-23
 * with is_2D): padded [n, h+2p, w+2p, c] -> out [n, h, w, c]; ep NULL or bn_mode 0: plain fold,
 * bn_mode 2: as cgan3d_reflect_fold_ex (slots: cgan3d_reflect_fold_slots(n, 1, h, w, c)) */
int cgan3d_reflect_fold2d(const float* padded, float* out, int32_t n, int32_t h, int32_t w, int32_t c,
                          int32_t pad, const cgan3d_epilogue* ep, void* stream);
/* reflect_fold with the epilogue's bn_mode-2 statistics of its output (other fields ignored);
 * slots of its slab: cgan3d_reflect_fold_slots() */
int32_t cgan3d_reflect_fold_slots(int32_t n, int32_t d, int32_t h, int32_t w, int32_t c);
int cgan3d_reflect_fold_ex(const float* padded, float* out, int32_t n, int32_t d, int32_t h,
                           int32_t w, int32_t c, int32_t pad, const cgan3d_epilogue* ep, void* stream);
int cgan3d_gp_interpolate(const float* real, const float* fake, const float* eps, float* out,
                          int32_t b, int64_t per_sample, void* stream);
/* The same with the reference's resampling when |real| != |fake| (model/utils.py:21-25): sample s
 * interpolates real row idx[s] and fake row idx[b + s] (idx: device int32 [2 b], drawn by the host);
 * real / fake hold n_real / n_fake rows and the kernel clamps every index into them (round 6: a bad
 * index can no longer read past either batch). */
int cgan3d_gp_interpolate_idx(const float* real, const float* fake, const int32_t* idx, const float* eps,
                              float* out, int32_t b, int64_t per_sample, int32_t n_real, int32_t n_fake,
                              void* stream);

int cgan3d_tanh_backward(const float* y, const float* dy, float* dz, int64_t n, void* stream);

/* --- patch loader (data/CCTADataLoader.py:88-104, data/Scaler.py:37-45): src = nvox interleaved
 *     (HU, label) pairs (src_dtype 0: int16, 1: float32), data = (HU - shift) / factor,
 *     seg = label != 0 --- */
int cgan3d_unpack_patches(const void* src, int32_t src_dtype, int64_t nvox, float shift, float factor,
                          float* data, uint8_t* seg, void* stream);
/* The same on at most max_blocks workgroups, four voxels per thread from 16-byte loads (src and data
 * 16-byte aligned, seg 4-byte aligned): src may be mapped host memory (cgan3d_host_alloc's *dev), so
 * the batch goes from the loader's pinned slot to its HBM tensors in this one launch. */
int cgan3d_unpack_patches_ex(const void* src, int32_t src_dtype, int64_t nvox, float shift, float factor,
                             float* data, uint8_t* seg, int32_t max_blocks, void* stream);
/* --- spatial augmentation (experiments/basic_conf.py:87-113: batchgenerators SpatialTransform_2,
 * augment_spatial_2 with random_crop=False; replaces the augmenter's per-sample numpy/scipy work).
 * data/seg: [n][a0][a1][a2] (C = 1), out of place into data_out/seg_out.  params (device, n x 16
 * floats per sample): A[9] row-major (rotation x scale applied to the zero-centred grid), ctr[3]
 * (patch centre, a/2 - 0.5), field slot (>= 0: elastic sample index into noise; -1: none;
 * -2: no transform drawn, copy), mag[3] (elastic magnitude + 1e-8 per axis).  noise (device,
 * n_elastic x 3 x a0*a1*a2): uniform [-1, 1) fields; gauss (device, n_elastic x 3 axes x
 * max(a0, a1, a2)): circular Gaussian kernels (the inverse DFT of scipy.ndimage.fourier_gaussian's
 * response).  data: cubic B-spline, mode 'nearest' (scipy.ndimage.map_coordinates order 3);
 * seg: nearest neighbour, 0 outside the patch (order 0, mode 'constant'). */
/* --- whole-scan inference (eval/CCTAContrastCorrector.py:60-81, patchly GridSampler + Aggregator
 * with averaging): add b patches [b][p0][p1][p2] at origins (b x 3 int32, device) into out[s0][s1][s2]
 * and 1 into weight (both zeroed by the caller); cgan3d_patch_normalize: out /= weight. */
int cgan3d_patch_accumulate(const float* patch, int32_t b, int32_t p0, int32_t p1, int32_t p2,
                            const int32_t* origins, float* out, float* weight, int32_t s0, int32_t s1, int32_t s2,
                            void* stream);
int cgan3d_patch_normalize(float* out, const float* weight, int64_t n, void* stream);
int64_t cgan3d_augment_ws_floats(int32_t n, int32_t a0, int32_t a1, int32_t a2, int32_t n_elastic);
int cgan3d_spatial_augment(const float* data, const uint8_t* seg, int32_t n, int32_t a0, int32_t a1, int32_t a2,
                           const float* params, const float* noise, int32_t n_elastic, const float* gauss,
                           float* data_out, uint8_t* seg_out, float* ws, void* stream);
/* batchgenerators MirrorTransform (experiments/conf_2D.py:36-43: axes (0, 1), p_per_sample 0.5;
 * augment_mirroring): data/seg [n][a0][a1][a2] out of place into data_out/seg_out, sample s flipped
 * along a_d where bit d of flags[s] (device, n int32) is set.  The host draws the flags. */
int cgan3d_mirror(const float* data, const uint8_t* seg, int32_t n, int32_t a0, int32_t a1, int32_t a2,
                  const int32_t* flags, float* data_out, uint8_t* seg_out, void* stream);

/* --- losses (model/loss.py:11-80, model/utils.py:12-41, Trainer.py:119-154) ---
 * losses[] slots: 0 D total, 1 W_D, 2 GP, 3 G (adversarial), 4 sim (ZNCC), 5 HU, 6 G-full. */
int64_t cgan3d_loss_ws_floats(int64_t n);
int cgan3d_critic_logits_grad(const float* logits, int32_t n_real, int32_t n_fake, int32_t n_gp,
                              int32_t per_sample, float gan_w, float* dlogits, float* losses,
                              void* stream);
int cgan3d_gradient_penalty(const float* grad, int32_t b, int64_t per_sample, float lambda_,
                            float* gamma_out, float* losses, float* ws, void* stream);
/* The same from per-sample partial sums of squares already made (part[s * chunks + c], e.g. by the
 * critic's first-layer input-grad with cgan3d_conv3d_sumsq_blocks): one scaling pass. */
int cgan3d_gradient_penalty_part(const float* grad, const float* part, int32_t b, int32_t chunks, int64_t per_sample,
                                 float lambda_, float* gamma_out, float* losses, const float* logits, int32_t n_real,
                                 int32_t n_fake, int32_t logit_ps, float gan_w, float* zero, int64_t zero_n,
                                 void* stream);
/* logits (optional, [real n_real x logit_ps | fake n_fake x logit_ps]): the same launch also writes the
 * Wasserstein term and the critic loss (what cgan3d_critic_logits_grad's losses would be), for a
 * caller whose dlogits are constant buffers written once (so that launch is not needed at all).
 * zero (optional, zero_n floats): written with zeros by the same launch — the critic's gradient arena
 * (optimizer_D.zero_grad, Trainer.py:109) without a fill launch of its own. */
/* dlogits may be NULL: the loss only (constant dlogits kept by the caller). */
int cgan3d_generator_logits_grad(const float* logits, int32_t n, float gan_w, float* dlogits,
                                 float* losses, void* stream);
int cgan3d_generator_output_grad(const float* opt_hat, const float* subopt, const float* att,
                                 const uint8_t* mask, const float* d_critic, int64_t n, float lo,
                                 float hi, float sim_w, float hu_w, float* dz_last, float* losses,
                                 float* ws, void* stream);

/* --- optimiser (torch.optim.Adam, experiments/basic_conf.py:55,67) ---
 * hyper (device): [lr, beta1, beta2, eps, step, weight_clip]; cgan3d_adam_tick increments step. */
int cgan3d_adam_tick(float* hyper, void* stream);
/* Zero `bytes` bytes of device memory (recorded in launch plans): the engine zeroes a network's
 * whole gradient arena once per update and then accumulates every layer's weight gradient
 * (CGAN3D_WGRAD_ACCUMULATE) — Trainer.py:109,146 optimizer.zero_grad. */
int cgan3d_zero(void* p, int64_t bytes, void* stream);
/* n <= 8 device-to-device copies of bytes[i] bytes from src[i] to dst[i] in one launch (host
 * arrays; a batch into the step's input slots).  Segments whose src or dst is not 16-byte aligned
 * are copied bytewise and limited to 4 KB (CGAN3D_EINVAL beyond). */
int cgan3d_copy_multi(const void* const* src, void* const* dst, const int64_t* bytes, int32_t n, void* stream);
/* The same with at most max_blocks workgroups (a copy out of mapped host memory, cgan3d_host_alloc,
 * running beside the step on a copy stream: a few blocks keep enough PCIe reads in flight). */
int cgan3d_copy_multi_ex(const void* const* src, void* const* dst, const int64_t* bytes, int32_t n,
                         int32_t max_blocks, void* stream);
/* Pinned host memory mapped into the device address space (hipHostMallocMapped): *host for the host
 * writer, *dev for kernels (cgan3d_copy_multi_ex, cgan3d_unpack_patches_ex).  Replaces the pinned
 * staging + non-blocking copy of the reference's batch upload (trainer/Trainer.py:165-167,182-183). */
int cgan3d_host_alloc(int64_t bytes, void** host, void** dev);
int cgan3d_host_free(void* host);

/* LayerNorm critic (experiments/gp_layernorm.py:9-11, model/blocks.py:40-45): per-sample
 * normalisation over (C, D, H, W) — one contiguous run of L floats per sample in NDHWC — without
 * affine parameters, then LeakyReLU; plus the forward-mode tangent and the adjoint it injects,
 * which the gradient penalty's double backward (model/utils.py:34-39) differentiates through.
 * cgan3d_ln_reduce writes per-sample partial sums (cgan3d_ln_partial_doubles doubles) of the
 * mode's quantities; cgan3d_ln_apply combines them per sample and runs the elementwise pass.
 * Formulas: csrc/ln.hip header.  All tensor pointers start at the slice's first sample. */
#define CGAN3D_LN_STATS 0 /* reduce: sum z, z^2            apply: a = lrelu(x^)                */
#define CGAN3D_LN_BWD 1   /* reduce: sum rho, rho x^        apply: dz (LayerNorm + lrelu backward) */
#define CGAN3D_LN_JVP 2   /* reduce: sum zdot, zdot x^      apply: adot (tangent)               */
#define CGAN3D_LN_SIG 3   /* reduce: sum da * adot          (no apply)                          */
#define CGAN3D_LN_ADJ 4   /* reduce: sum xbar, xbar x^      apply: zbar (primal adjoint)        */
typedef struct cgan3d_ln_args {
  int32_t n;        /* samples */
  int32_t mode;
  int64_t L;        /* elements per sample */
  float slope, eps; /* LeakyReLU slope, LayerNorm eps (1e-5) */
  const float* z;   /* conv output (pre-norm) [n][L] */
  const float* da;  /* dL/d(activation) [n][L] (BWD, SIG, ADJ) */
  const float* zdot;  /* tangent conv output (JVP, ADJ) */
  const float* adot;  /* tangent activation (SIG) */
  const float* abar;  /* primal adjoint of the activation (ADJ; NULL = 0) */
  const double* p_stats, *p_bwd, *p_jvp, *p_sig, *p_adj; /* partials of the modes */
} cgan3d_ln_args;
int64_t cgan3d_ln_partial_doubles(int32_t n, int64_t L);
int cgan3d_ln_reduce(const cgan3d_ln_args* args, double* partials, void* stream);
int cgan3d_ln_apply(const cgan3d_ln_args* args, float* out, void* stream);
int cgan3d_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                const float* hyper, void* stream);

/* --- launch plans (the step engine's replacement for a replayed hipGraph; Trainer.py:163-203 is
 * the sequence recorded) ---
 * Between cgan3d_plan_begin and cgan3d_plan_end every entry point called on this host thread
 * RECORDS what it would enqueue (kernel launches with by-value arguments, workspace memsets,
 * cgan3d_stream_wait) instead of enqueuing it; operand checks still run at record time.
 * cgan3d_plan_run re-issues the recorded sequence on the recorded streams (one host call for a
 * whole step).  Every buffer a recorded launch touches must keep its address while the plan lives. */
int cgan3d_plan_begin(void);
int cgan3d_plan_end(void** plan);
int64_t cgan3d_plan_size(void* plan);
int cgan3d_plan_run(void* plan);
int cgan3d_plan_destroy(void* plan);
/* Round 6, measurement: launches of kernels whose (mangled) name contains `substring` (or one of several
 * separated by '|'), recorded while
 * it is set (NULL or "" clears it; per host thread), are issued with their own start / stop timing
 * events (hipExtLaunchKernel); after a cgan3d_plan_run and a synchronisation, cgan3d_plan_times writes
 * each timed launch's duration in ms (up to `max`, in record order) and returns how many there are. */
int cgan3d_plan_time_filter(const char* substring);
int64_t cgan3d_plan_times(void* plan, float* ms, int64_t max);
/* The same launches as a timeline of the last run: start / end in ms from the first timed launch's start,
 * and the stream of each (index in order of first appearance); cgan3d_plan_timed_name(plan, i) is the
 * mangled kernel name of launch i.  (A kernel trace without a profiler: rocprofv3's per-dispatch cost
 * makes the host issue the bottleneck of a traced plan step.) */
int64_t cgan3d_plan_timeline(void* plan, float* start_ms, float* end_ms, int32_t* stream_id, int64_t max);
const char* cgan3d_plan_timed_name(void* plan, int64_t i);
/* `waiter` waits for all work enqueued so far on `signaler` (recorded when inside a plan). */
int cgan3d_stream_wait(void* waiter, void* signaler);

/* ---- data-parallel gradient averaging (RCCL over xGMI), SURVEY.md §8e.  Replaces the gradient
 * all-reduce DDP would issue around optimizer_D.step() / optimizer_G.step() (Trainer.py:135,157):
 * the reference itself runs on one device.  `comm` is an ncclComm_t: either the caller's own
 * (torch.distributed's, when cgan3d_comm_shared_library() == 1, i.e. the entry points resolve to
 * the RCCL the process has already loaded — the default, one communicator per process), or one
 * of this library's: rank 0 creates the unique id (cgan3d_comm_id_bytes() bytes), the caller
 * broadcasts it, every rank calls cgan3d_comm_init.  cgan3d_allreduce_mean averages n fp32 in
 * place on `stream` and is recorded into a launch plan like a kernel launch (cgan3d_plan_*), so a
 * data-parallel step replays as one plan. */
int32_t cgan3d_comm_shared_library(void);
int32_t cgan3d_comm_id_bytes(void);
int cgan3d_comm_unique_id(void* out);
int cgan3d_comm_init(const void* unique_id, int32_t nranks, int32_t rank, void** comm);
int cgan3d_comm_destroy(void* comm);
int cgan3d_allreduce_mean(void* comm, float* buf, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CGAN3D_H_ */
