/*
 * fedagg.h — C-ABI of the MI355X (gfx950) server-side aggregation library
 * (libfedagg.so, built from fedsim_amd/csrc/fedagg_kernels.hip).
 *
 * This is the drop-in boundary for FedSim's server aggregation hot path.
 * The reference has no native code: each entry point replaces a piece of
 * PyTorch-CPU arithmetic that the reference runs in Python.
 *
 *   fedagg_reduce_f32 / fedagg_reduce_rows_f32
 *       replaces SerialAggregator.add            fedsim/utils/aggregators.py:17-40
 *       (value*weight then sum_v+new_v, once per client, called from
 *        serial_aggregation fedsim/distributed/centralized/training/utils.py:45-46)
 *       and, with FEDAGG_FINALIZE, SerialAggregator.get/pop's  v / w
 *                                                  fedsim/utils/aggregators.py:56-60,118-122
 *   fedagg_reduce_blocked_f32
 *       same, over a column-blocked HBM slab layout
 *   fedagg_finalize_f32 / fedagg_finalize_f64
 *       replaces SerialAggregator.get/pop's v / w  fedsim/utils/aggregators.py:56-60,118-122
 *   fedagg_reduce_rows_ref
 *       SerialAggregator.add on bf16 / fp16 / fp64 tensor keys, the reference's
 *       rounding per product and per add                  aggregators.py:17-40
 *   fedagg_fedavg_sgd_f32
 *       replaces FedAvg.optimize's pseudo-grad + torch.optim.SGD.step
 *                                                  fedsim/distributed/centralized/training/fedavg.py:199-203
 *   fedagg_adabest_sgd_f32
 *       replaces AdaBest.optimize's h / new_params / pseudo-grad + SGD.step
 *       + avg_params write-back                    fedsim/distributed/centralized/training/adabest.py:178-188
 *   fedagg_feddyn_sgd_f32
 *       replaces FedDyn.optimize's h update, new_params, pseudo-grad + SGD.step
 *                                                  fedsim/distributed/centralized/training/feddyn.py:169-194
 *   fedagg_server_step_f32
 *       the three optimize epilogues above with any torch.optim.SGD
 *       configuration (momentum / nesterov / weight decay / maximize)
 *   fedagg_reduce_step_blocked_f32 / fedagg_reduce_step_rows_f32
 *       SerialAggregator.pop + optimize fused: the round's last drain and the
 *       server step in one pass              aggregators.py:104-122 + fedavg.py:193-208
 *
 * Bit-exactness contract (exact mode, the default): every output equals the
 * reference CPU aggregation bit for bit, given the same arrival order:
 *     acc_0 = +0.0f ;  acc_{k+1} = fl32(acc_k + fl32(x_k * w_k))      (no FMA)
 *     avg   = fl32(acc_K / W)                                        (true division)
 * where w_k = fl32(python weight) and W = fl32(python sum of raw weights).
 *
 * Conventions
 *   - All pointers are device pointers (HBM) unless stated; all buffers are
 *     owned by the caller; the library allocates nothing and keeps no state.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *     Every call is asynchronous and stream-ordered.
 *   - Return value: 0 on success, a positive hipError_t code if a HIP call
 *     failed, or a negative FEDAGG_E* code for a rejected argument.
 *     Nothing throws across the ABI.
 */
#ifndef FEDAGG_H_
#define FEDAGG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 1: round-1 reduce / pack / step entry points; 2: + the FedDF teacher
   (linear, conv2d, pad-LRN-maxpool) and slab-row (pack_segments, unpack_row)
   entry points and their structs; 3: flag bits 0x10000 / 0x20000 (the
   flat-load and LDS-weight A/B switches, measured and rejected) are no
   longer accepted (FEDAGG_EINVAL); 4: + fedagg_finalize_f64 and
   fedagg_reduce_rows_ref (the dtype-generic SerialAggregator's fp64 / bf16 /
   fp16 keys); 5: + fedagg_rows_plan; 6: + fedagg_host_mapped (page-locked
   host operands read and written in place) */
#define FEDAGG_ABI_VERSION 6

/* flags for the reduce entry points */
#define FEDAGG_INIT      0x1  /* ignore acc_in: start from +0.0f (first batch of a round) */
#define FEDAGG_FINALIZE  0x2  /* store fl32(acc / W32) instead of the raw sum              */
#define FEDAGG_NT        0x4  /* non-temporal (streaming) loads of the client rows         */
#define FEDAGG_SCALAR    0x8  /* force the 4-byte-per-lane path (rows not 16-B aligned)    */
/* bits 8..11: k-unroll selector, 0 = library default, 1 = 4, 2 = 8, 3 = 16, 4 = 2,
 * 5 = 32 (narrow mapping only; it takes 2 / 3 / 5, anything else = default 16) */
#define FEDAGG_UNROLL_SHIFT 8
#define FEDAGG_UNROLL_MASK  0xF00
/* bits 12..13: float4 slots per lane, 0 = library default, 1 = 1, 2 = 2, 3 = 4 */
#define FEDAGG_VPT_SHIFT 12
#define FEDAGG_VPT_MASK  0x3000
/* bits 14..15: workgroup size for the blocked layout, 0 = default, 1 = 256,
 * 2 = 512, 3 = 1024 lanes (float4 slots per lane = C / (4 * lanes)) */
#define FEDAGG_BS_SHIFT 14
#define FEDAGG_BS_MASK  0xC000
/* bits 16..17 are reserved (rejected).  The blocked layout reads through
 * buffer descriptors, and falls back to flat global loads by itself when a
 * column block's region is >= 4 GiB; per-client weights are wave-uniform
 * scalar loads. */
/* bits 18..20: column mapping of the reduce kernels.  An in-order per-column
 * sum is parallel over columns only, so at small P the f32x4-slot ("wide")
 * kernels leave CUs idle (P = 199,210 is 778 waves).  0 = library default
 * (narrow: one column per lane below P = 2^20, two from there on, four for
 * P >= 2^24 with at most 64 rows per call), 1 = wide
 * (f32x4 slots; the unroll / VPT / BS tuning bits apply to it), 2 / 3 / 4 =
 * narrow with one / two / four columns per lane (each workgroup one wave;
 * falls back to fewer columns when P or an operand's alignment does not
 * allow them).  Same results. */
#define FEDAGG_MAP_SHIFT 18
#define FEDAGG_MAP_MASK  0x1C0000
/* FAST (reordered) mode: when P is too small for one column per lane to fill
 * the chip (below 65,536 columns), split the K rows of each 64-column tile over
 * up to 16 waves of a workgroup (per-client weights staged in LDS, fmaf partial
 * sums combined through LDS in a fixed order).  Deterministic, but NOT the
 * reference's summation order: parity is normwise (<= 1e-6 relative and the
 * gamma_K forward-error bound), not bitwise.  Ignored (exact kernels) where it
 * would not add parallelism. */
#define FEDAGG_FAST     0x200000
/* fedagg_teacher_linear_f32: apply ReLU to the layer's output (a following
 * torch.relu / nn.ReLU fused into the layer) */
#define FEDAGG_RELU     0x400000
/* fedagg_teacher_conv2d_f32: take the im2col-gather kernel even where the
 * LDS-resident one applies (A/B and its own tests; same results up to the
 * chain order fedagg_conv_order reports) */
#define FEDAGG_CONV_GATHER 0x800000
/* fedagg_teacher_conv2d_f32: the 2 x 2 / stride 2 max pool that follows the
 * layer (after its ReLU) fused into the store, padding 0, or 1 with
 * FEDAGG_CONV_POOL_PAD1 (SimpleCNN's F.max_pool2d(x, 2, 2, padding=1),
 * simple_models.py:156-159): y is then [K, M, OC, PH, PW], PH = (OH + 2p -
 * 2) / 2 + 1 (PW alike), max over each window's members inside the conv
 * output (-inf padding), NaN propagating, in window order -- the same bits as
 * the conv followed by fedagg_pad_lrn_maxpool_f32 with that pool.  Only for
 * the shapes fedagg_conv_pool_fusable accepts (else FEDAGG_EINVAL). */
#define FEDAGG_CONV_MAXPOOL2  0x2000000
#define FEDAGG_CONV_POOL_PAD1 0x4000000

/* negative error codes */
#define FEDAGG_EINVAL   (-22) /* bad size / null pointer / bad flag combination */
#define FEDAGG_EALIGN   (-23) /* internal: misaligned pointer passed to an aligned-only path */

/* Version of this ABI (FEDAGG_ABI_VERSION). */
int fedagg_abi_version(void);

/* Human-readable message for a return code (static storage, never NULL). */
const char* fedagg_strerror(int code);

/*
 * Which reduce kernel a call with these flags takes for B rows x P columns
 * (host-side decision, no device access): *vw = columns per lane of the
 * narrow mapping (1, 2 or 4), or 0 for the wide f32x4-slot kernels; *unroll =
 * the narrow kernel's k-unroll (0 when wide).  max_vw (1, 2 or 4): the most
 * columns per lane P and the operands' alignment allow.
 */
int fedagg_column_mapping(int64_t P, int64_t B, int flags, int max_vw, int* vw, int* unroll);

/*
 * Weighted sequential reduction of B client rows into one accumulator.
 *
 *   X       row-major [B, ldx] fp32 slab; row k holds client k's flat params
 *           (layout of vectorize_module, fedsim/utils/convert_parameters.py:78-94).
 *           A parameter shard is addressed as X + offset with the same ldx.
 *   ldx     row pitch in elements (>= P)
 *   w       [B] fp32 per-client weights, already rounded to fp32
 *   B, P    number of rows (B >= 0) and columns (P >= 0)
 *   acc_in  [P] running sum from earlier batches (ignored with FEDAGG_INIT)
 *   out     [P] destination; may alias acc_in
 *   W32     fp32 total weight, used only with FEDAGG_FINALIZE
 *
 * For every column p, rows are consumed in order k = 0..B-1, so chaining
 * batches through acc_in/out keeps the reference's arrival order.
 * B == 0 with FEDAGG_INIT writes zeros (or 0/W32 when finalizing).
 */
int fedagg_reduce_f32(const float* X, int64_t ldx, const float* w, int64_t B,
                      int64_t P, const float* acc_in, float* out, float W32,
                      int flags, void* stream);

/*
 * Same reduction, but row k lives at rows[k] (a device array of B device
 * pointers, each to P contiguous fp32).  Lets the caller reduce client tensors
 * already resident in HBM without packing them into a slab first.
 * The table lives in device memory and is not inspected on the host: the
 * caller must pass FEDAGG_SCALAR unless every rows[k] is 16-byte aligned.
 * With no tuning field set (FEDAGG_MAP/UNROLL/VPT/BS_MASK all zero) and
 * 16-byte operands, large P takes the wide per-row tiles; any tuning field
 * selects the narrow / wide column kernels those bits name.
 */
int fedagg_reduce_rows_f32(const float* const* rows, const float* w, int64_t B,
                           int64_t P, const float* acc_in, float* out, float W32,
                           int flags, void* stream);

/*
 * Which kernel fedagg_reduce_rows_f32 launches for B rows x P columns under
 * ``flags`` when every operand is 16-byte aligned (aligned16 != 0) or not
 * (host-side decision, no device access): *kind = one of FEDAGG_ROWS_*.
 */
#define FEDAGG_ROWS_NARROW1 1 /* one column per lane                        */
#define FEDAGG_ROWS_NARROW2 2 /* two columns per lane                       */
#define FEDAGG_ROWS_NARROW4 3 /* four columns per lane                      */
#define FEDAGG_ROWS_WIDE    4 /* f32x4-slot column kernels (FEDAGG_MAP = 1) */
#define FEDAGG_ROWS_TILE4x8 5 /* wide per-row tile, 4 rows x 8 KiB          */
#define FEDAGG_ROWS_TILE8x4 6 /* wide per-row tile, 8 rows x 4 KiB          */
#define FEDAGG_ROWS_SPLITK  7 /* FEDAGG_FAST split-K (small P, reordered)   */
#define FEDAGG_ROWS_FLAT    8 /* P * 4 >= 4 GiB: flat loads                 */
int fedagg_rows_plan(int64_t P, int64_t B, int flags, int aligned16, int* kind);

/*
 * Same reduction over a COLUMN-BLOCKED slab: columns are cut into blocks of C
 * floats (C = 1024, 2048 or 4096, one workgroup's span) and, inside a block,
 * the Kcap rows are contiguous:  element (k, p) is at
 *     Xb[((p / C) * Kcap + k) * C + (p % C)],   Xb sized ceil(P / C) * Kcap * C.
 * Each workgroup then streams one contiguous region instead of K strided
 * 100-MB-apart rows.  Rows 0..B-1 (B <= Kcap) are reduced; rows r0..r0+B-1
 * of a slab are reduced by passing Xb + r0*C (same Kcap), which is how a ring
 * of client rows is drained in arrival order.
 */
int fedagg_reduce_blocked_f32(const float* Xb, int64_t Kcap, int64_t C, const float* w,
                              int64_t B, int64_t P, const float* acc_in, float* out,
                              float W32, int flags, void* stream);

/*
 * FedDF's teacher ensemble (fedsim/distributed/centralized/training/feddf.py
 * :117-122 runs every client model on each distillation batch): ONE nn.Linear
 * layer of K stacked teacher models, on the matrix cores (f32 in / f32
 * accumulate):
 *   y[k][m][n] = act(sum_i x[k*x_kstride + m*in + i] * W_k[n][i] + b_k[n])
 * W_k = params + k*params_kstride + w_off ([out, in] row-major, the teacher's
 * flat vector in parameters_to_vector order); b_k = params + k*params_kstride
 * + b_off (b_off = -1: no bias).  x_kstride = 0 shares one input across the
 * teachers (the batch itself).  y is [K, M, out] contiguous.  flags:
 * FEDAGG_RELU.  Results are exact f32 k-ordered fmaf chains (the bias added
 * last): normwise, not bitwise, equal to a CPU / BLAS Linear.
 */
int fedagg_teacher_linear_f32(const float* x, int64_t x_kstride, const float* params,
                              int64_t params_kstride, int64_t w_off, int64_t b_off, int64_t K,
                              int64_t M, int64_t in, int64_t out, float* y, int flags,
                              void* stream);

/*
 * FedDF's teacher ensemble, convolutional layers (the same feddf.py:117-122
 * forwards; fedsim/models/simple_models.py:156-158, 245-249 are the
 * reference's nn.Conv2d layers): ONE nn.Conv2d (groups 1, dilation 1, zero
 * padding) of K stacked teachers as an implicit GEMM on the matrix cores
 * (v_mfma_f32_32x32x2_f32):
 *   y[k][m][oc][oh][ow] = act(b_k[oc] + sum_{c,kh,kw} W_k[oc][c][kh][kw] *
 *                             x_k[m][c][oh*stride_h - pad_h + kh][ow*stride_w - pad_w + kw])
 * with out-of-range input positions reading 0 (bottom / right padding is
 * implied by OH / OW, so torch's asymmetric padding="same" for even kernels
 * fits).  x_k = x + k*x_kstride ([M, C, H, W] contiguous; x_kstride = 0: one
 * input shared by all teachers); W_k = params + k*params_kstride + w_off
 * ([OC, C, KH, KW] row-major, the teacher's flat vector); b_off = -1: no
 * bias.  y is [K, M, OC, OH, OW] contiguous.  flags: FEDAGG_RELU,
 * FEDAGG_CONV_GATHER, FEDAGG_CONV_MAXPOOL2 (| FEDAGG_CONV_POOL_PAD1).
 * Each output is an exact f32 fmaf chain from +0.0f,
 * then one bias add: normwise, not bitwise, equal to a CPU conv.  The chain's
 * order is what fedagg_conv_order reports for the shape:
 *   0  (the im2col-gather kernel, and the LDS-resident kernel for C = 1 or 3
 *      with every channel staged at once): r = (c, kh, kw) in order, an odd
 *      count closed by one fmaf(0, 0, acc) term;
 *   cc (the LDS-resident kernel: stride 1, KH = KW = 3 or 5): channel chunks
 *      of cc, then kh, then channel pairs, then kw, then the pair's two
 *      channels; channels past C are fmaf(0, 0, acc) terms.
 */
typedef struct fedagg_conv2d_shape {
  int64_t M, C, H, W;          /* per-teacher input [M, C, H, W]            */
  int64_t OC, KH, KW;          /* output channels, kernel size              */
  int64_t stride_h, stride_w;  /* >= 1                                      */
  int64_t pad_h, pad_w;        /* top / left zero padding                   */
  int64_t OH, OW;              /* output size                               */
} fedagg_conv2d_shape;

int fedagg_teacher_conv2d_f32(const float* x, int64_t x_kstride, const float* params,
                              int64_t params_kstride, int64_t w_off, int64_t b_off, int64_t K,
                              const fedagg_conv2d_shape* shape, float* y, int flags,
                              void* stream);

/* Reductions per LDS stage the conv kernel takes for R = C*KH*KW (16 or 32;
 * the exact chain is the same either way). Host-side, no device access. */
int fedagg_conv_stage(int64_t R);

/* 1 if fedagg_teacher_conv2d_f32 fuses the max pool FEDAGG_CONV_MAXPOOL2 (|
 * FEDAGG_CONV_POOL_PAD1) asks for on this shape (the LDS-resident kernel for
 * C = 1 or 3, stride 1, 3 x 3 / 5 x 5), else 0. Host-side, no device access. */
int fedagg_conv_pool_fusable(const fedagg_conv2d_shape* shape, int flags);

/* Chain order of fedagg_teacher_conv2d_f32 for this shape and flags: 0 for
 * the (c, kh, kw) order, else the channel chunk cc (see above). Host-side. */
int fedagg_conv_order(const fedagg_conv2d_shape* shape, int flags);

/*
 * The memory-bound chain after a convolution of the reference's CNNs
 * (simple_models.py:246-248, 250-252: F.pad(x, (0, 1, 0, 1)) ->
 * F.local_response_norm(size 4, alpha 1e-3/9) -> F.max_pool2d(3, 2); :157,
 * :159 max_pool2d(2, 2, padding 1)) in ONE pass over x [N, C, H, W]:
 *   1. zero padding (pad_top / bottom / left / right, F.pad's constant 0);
 *   2. lrn_size > 0: local_response_norm across channels with ATen's
 *      roundings (window [c - size/2, c + (size-1)/2], zeros outside):
 *      s = sum fl32(x*x) in channel order from +0, avg = s / size,
 *      d = powf(fl32(fl32(avg * alpha) + k), beta), v = x / d;
 *   3. pool_kh > 0: max_pool2d (kernel pool_kh x pool_kw, stride pool_sh x
 *      pool_sw, implicit -inf padding pool_ph / pool_pw <= half the kernel,
 *      floor mode, NaN propagates).  pool_kh = 0: no pooling.
 * Zero padding and LRN commute (LRN(0) = 0), so pad -> LRN and LRN -> pad
 * are both this call.  y is [N, C, OH, OW] contiguous; fedagg_pool_output
 * gives OH / OW (and the channels per workgroup / LDS block).
 * flags: 0, or FEDAGG_POOL_PLANES to take the per-block kernels (each
 * workgroup re-reads its block's LRN halo) instead of the sliding channel
 * window for planes of <= 1024 positions; the results are the same bits.
 */
#define FEDAGG_POOL_PLANES 0x1000000
typedef struct fedagg_pool_args {
  int64_t N, C, H, W;
  int64_t pad_top, pad_bottom, pad_left, pad_right;
  int64_t lrn_size;
  float lrn_alpha, lrn_beta, lrn_k;
  int32_t flags;
  int64_t pool_kh, pool_kw, pool_sh, pool_sw, pool_ph, pool_pw;
} fedagg_pool_args;

int fedagg_pool_output(const fedagg_pool_args* args, int64_t* OH, int64_t* OW, int64_t* CB);

int fedagg_pad_lrn_maxpool_f32(const float* x, const fedagg_pool_args* args, float* y,
                               void* stream);

/*
 * vectorize_module straight into a slab row (fedsim/utils/convert_parameters.py
 * :78-94, parameters_to_vector + the clone at training/utils.py:34): write
 * the concatenation of nseg device segments into row r of a column-blocked
 * slab [ceil(P/C), Kcap, C] in one launch.  segs is a DEVICE array of nseg
 * int64 triples {source pointer, first column, length > 0}, sorted by first
 * column and tiling [0, P) exactly (a model's parameters in registration
 * order; adjacent parameters that are adjacent in memory may be one segment).
 * Xb must be 16-byte aligned.
 */
int fedagg_pack_segments_f32(const int64_t* segs, int64_t nseg, int64_t P, float* Xb,
                             int64_t Kcap, int64_t C, int64_t r, void* stream);

/*
 * Row r of a column-blocked slab copied out to P contiguous fp32 at dst (both
 * 16-byte aligned device memory): a slab row read back as a flat vector.
 */
int fedagg_unpack_row_f32(const float* Xb, int64_t Kcap, int64_t C, int64_t r, int64_t P,
                          float* dst, void* stream);

/*
 * Pack one client vector (P contiguous fp32, host-pinned or device memory)
 * into row r of a column-blocked slab [ceil(P/C), Kcap, C]: a copy kernel
 * for 16-byte aligned device memory and for page-locked host memory mapped
 * at its own address (read in place over PCIe), else one 2-D DMA.
 * This is the HBM side of SerialAggregator.add's snapshot (the reference's
 * clone at fedsim/distributed/centralized/training/utils.py:34) and of
 * vectorize_module's packing (fedsim/utils/convert_parameters.py:78-94).
 */
int fedagg_pack_row_f32(const float* src, int64_t P, float* Xb, int64_t Kcap, int64_t C,
                        int64_t r, void* stream);

/*
 * 1 if [p, p + nbytes) is page-locked host memory the GPU reaches at the
 * host address itself (hipHostMalloc on this platform: torch's pin_memory),
 * else 0 (pageable or device memory, or mapped at another address).  Such
 * memory may stand in for device memory as a pack source and as a server
 * step's operands (struct fedagg_step_args, fedagg_server_step_f32): the
 * kernels then read and write it in place over PCIe, with no DMA to issue --
 * the host-resident server state of FedSim's device="cpu" runs.
 */
int fedagg_host_mapped(const void* p, int64_t nbytes);

/* out[p] = fl32(acc[p] / W32)  (IEEE true division; out may alias acc). */
int fedagg_finalize_f32(const float* acc, float W32, int64_t P, float* out,
                        void* stream);

/*
 * out[p] = acc[p] / W  in f64 (IEEE true division; out may alias acc).
 * SerialAggregator.get/pop's  v / w  for an fp64 sum (aggregators.py:56-60,
 * 118-122): ATen's CPU true division by a Python scalar is a / (double)w,
 * while torch's HIP kernel multiplies by the reciprocal, which is not the
 * reference's rounding.  Bf16 / fp16 / integer sums divide in f32
 * (fedagg_finalize_f32 on the converted sum, as ATen's opmath does).
 */
int fedagg_finalize_f64(const double* acc, double W, int64_t P, double* out,
                        void* stream);

/*
 * The reference's SerialAggregator arithmetic on bf16 / fp16 / fp64 rows
 * (aggregators.py:17-40 for a key whose values are such tensors: an fp64 or
 * bf16 model).  ATen rounds every ``value * weight`` and every ``sum + new``
 * to the dtype (computing in float, its opmath type, for bf16 / fp16; in
 * double for fp64), so per column, in arrival order:
 *     s_1 = rnd(rnd(x_0 * w_0) + 0),   s_{k+1} = rnd(s_k + rnd(x_k * w_k))
 * rows: DEVICE table of B pointers to P elements of the dtype; w: B DEVICE
 * weights, float (fl32 of the Python weight) for BF16 / F16, double for F64;
 * acc_in: the running sum s_k (ignored with FEDAGG_INIT, which starts the
 * chain with the first row); out may alias acc_in.  flags: FEDAGG_INIT,
 * FEDAGG_SCALAR (some row not 16-B aligned: element loads only).  Bitwise
 * equal to the reference's CPU tensors.
 */
#define FEDAGG_DTYPE_BF16 1
#define FEDAGG_DTYPE_F16  2
#define FEDAGG_DTYPE_F64  3
int fedagg_reduce_rows_ref(int dtype, const void* const* rows, const void* w, int64_t B,
                           int64_t P, const void* acc_in, void* out, int flags, void* stream);

/*
 * FedAvg server step with plain SGD (no momentum / weight decay / nesterov):
 *   g        = fl32(cloud - avg)
 *   cloud'   = fma(-lr32, g, cloud)         (torch CPU SGD.step's add_(alpha=-lr))
 * If grad_out != NULL the pseudo-gradient g is stored there too.
 */
int fedagg_fedavg_sgd_f32(const float* avg, float lr, float* cloud,
                          float* grad_out, int64_t P, void* stream);

/*
 * AdaBest server step with plain SGD:
 *   h        = fl32(beta32 * fl32(avg_prev - avg))
 *   new      = fl32(avg - h)
 *   g        = fl32(cloud - new)
 *   cloud'   = fma(-lr32, g, cloud)
 *   avg_prev'= avg
 */
int fedagg_adabest_sgd_f32(const float* avg, float beta, float lr, float* cloud,
                           float* avg_prev, float* grad_out, int64_t P,
                           void* stream);

/*
 * FedDyn server step with plain SGD
 * (fedsim/distributed/centralized/training/feddyn.py:169-194):
 *   g1       = fl32(cloud - avg)
 *   h'       = fl32(h + fl32(ratio32 * g1))      ratio32 = fl32(weight / num_clients)
 *   new      = fl32(avg - h')
 *   g        = fl32(cloud - new)
 *   cloud'   = fma(-lr32, g, cloud)
 *   avg_prev'= avg   (if avg_prev != NULL)
 */
int fedagg_feddyn_sgd_f32(const float* avg, float ratio, float lr, float* cloud, float* h,
                          float* avg_prev, float* grad_out, int64_t P, void* stream);

/*
 * General fused server step: an algorithm's pseudo-gradient followed by the
 * full torch.optim.SGD update (momentum, dampening, nesterov, weight decay,
 * maximize) with ATen's roundings (torch/optim/sgd.py _single_tensor_sgd, the
 * path torch takes for CPU params):
 *   d   = maximize ? -g : g
 *   d   = fma(param, wd, d)                          if wd != 0
 *   buf = init ? d : fma(d, 1-damp, fl32(buf * m))   if m != 0
 *   d   = nesterov ? fma(buf, m, d) : buf            if m != 0
 *   param = fma(d, -lr, param)
 * g per algo:
 *   FEDAGG_ALGO_FEDAVG   g = cloud - avg                        (fedavg.py:199)
 *   FEDAGG_ALGO_ADABEST  g = cloud - (avg - coef*(aux - avg)),  aux <- avg
 *                        coef = beta, aux = avg_params          (adabest.py:178-188)
 *   FEDAGG_ALGO_FEDDYN   aux <- aux + coef*(cloud - avg); g = cloud - (avg - aux);
 *                        avg_prev <- avg (if non-NULL)
 *                        coef = weight/num_clients, aux = h     (feddyn.py:176-192)
 * The scalars in *sgd are the fp32 values ATen computes with: each is the
 * Python double rounded once (neg_lr = fl32(-lr), one_minus_dampening =
 * fl32(1 - dampening)).  momentum_init != 0 means the optimizer has no
 * momentum buffer yet (torch clones d into it).  grad_out receives g.
 */
#define FEDAGG_ALGO_FEDAVG  0
#define FEDAGG_ALGO_ADABEST 1
#define FEDAGG_ALGO_FEDDYN  2

typedef struct fedagg_sgd_params {
  float neg_lr;
  float momentum;
  float one_minus_dampening;
  float weight_decay;
  int nesterov;
  int maximize;
} fedagg_sgd_params;

int fedagg_server_step_f32(int algo, const float* avg, float coef, float* cloud, float* aux,
                           float* avg_prev, float* momentum_buf, int momentum_init,
                           float* grad_out, const fedagg_sgd_params* sgd, int64_t P,
                           void* stream);

/*
 * The operands of one server step, for the fused reduce + step entry below.
 * Same meaning as the fedagg_server_step_f32 arguments; avg_out (optional)
 * additionally receives the average itself.
 */
typedef struct fedagg_step_args {
  int algo;               /* FEDAGG_ALGO_*                                     */
  float coef;             /* AdaBest beta / FedDyn weight/num_clients          */
  float* cloud;           /* [P] in/out, required                              */
  float* aux;             /* [P] in/out: AdaBest avg_params / FedDyn h         */
  float* avg_prev;        /* [P] out, FedDyn only, optional                    */
  float* momentum_buf;    /* [P] in/out, required iff sgd.momentum != 0        */
  int momentum_init;      /* != 0: no momentum buffer yet (buf <- d)           */
  float* grad_out;        /* [P] out, optional: the pseudo-gradient g          */
  float* avg_out;         /* [P] out, optional: the average                    */
  fedagg_sgd_params sgd;
} fedagg_step_args;

/*
 * The last drain of a round fused with the server step:
 *     fedagg_reduce_blocked_f32(..., out = avg)  then  fedagg_server_step_f32(avg, ...)
 * in ONE pass over the slab. The average never round-trips through HBM.
 * It replaces SerialAggregator.pop (aggregators.py:104-122) followed by the
 * algorithm's optimize (fedavg.py:193-208, adabest.py:172-189,
 * feddyn.py:157-194), with bit-identical results to the two-call sequence.
 * Flags: FEDAGG_INIT / FEDAGG_FINALIZE as for the reduce; the column-mapping
 * bits and, for the narrow mapping, the unroll selector apply (the wide
 * mapping uses its per-C default configuration, non-temporal loads).
 * FEDAGG_SCALAR is rejected. Every [P] operand must be 16-byte aligned, and a
 * column block's region (Kcap * C * 4 bytes) must be < 4 GiB.
 */
int fedagg_reduce_step_blocked_f32(const float* Xb, int64_t Kcap, int64_t C, const float* w,
                                   int64_t B, int64_t P, const float* acc_in, float W32,
                                   int flags, const fedagg_step_args* step, void* stream);

/*
 * The same fused last drain + server step over client rows that stay where
 * the caller's tensors live (rows[k]: a device array of B device pointers,
 * each to P contiguous, 16-byte aligned fp32), i.e. fedagg_reduce_rows_f32
 * followed by fedagg_server_step_f32 in one pass.  This is the zero-copy
 * round of HBM-resident client vectors (GPU-local training): no pack, no
 * slab; SerialAggregator.add (aggregators.py:23-40) only records the row.
 * Flags as for fedagg_reduce_step_blocked_f32.  FEDAGG_NT is read only by
 * the wide mapping (FEDAGG_MAP_WIDE); the narrow mappings (the default at
 * every P) and the flat path of rows >= 2^30 columns always load the client
 * rows non-temporally (measured +4.7 % at 1000 x 25 M).
 */
int fedagg_reduce_step_rows_f32(const float* const* rows, const float* w, int64_t B,
                                int64_t P, const float* acc_in, float W32, int flags,
                                const fedagg_step_args* step, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_H_ */
