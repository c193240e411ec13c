// fedagg_kernels.hip — MI355X (gfx950 / CDNA4) kernels for FedSim's server
// aggregation hot path, exported through the C-ABI in include/fedagg.h.
//
// What the reference does (pure Python + PyTorch CPU):
//   serial_aggregation   fedsim/distributed/centralized/training/utils.py:34-46
//     -> SerialAggregator.add  fedsim/utils/aggregators.py:23-40
//        new_v = value * weight          (fp32 tensor x Python scalar -> fl32(w))
//        sum_v = sum_v + new_v           (starts from the int 0)
//   SerialAggregator.pop  fedsim/utils/aggregators.py:104-122  -> v / w
//   FedAvg.optimize       fedsim/distributed/centralized/training/fedavg.py:193-208
//   AdaBest.optimize      fedsim/distributed/centralized/training/adabest.py:172-189
//
// Design (MI355X-first, not a translation — the reference has no kernels):
//   * The reduction is HBM-bound (0.5 flop/byte, no MFMA).  Every client row is
//     streamed exactly once: each lane owns a few columns and walks the K
//     client rows in arrival order; the running sum never leaves VGPRs.
//   * Columns are the only parallelism an in-order sum has, so how many a lane
//     owns decides whether the chip fills: the default "narrow" kernels
//     (k_reduce_narrow) give each lane 1, 2 or 4 adjacent columns (256 B, 512 B
//     or 1 KiB per wave-instruction), the "wide" ones (k_reduce_vec) VPT f32x4
//     slots.  The library picks per call (fedagg_column_mapping); see
//     DESIGN.md §3 for the measurements behind the choice.
//   * Exact mode keeps the reference's per-column order k = 0..K-1 and its
//     rounding (separate mul and add, no contraction, IEEE true division), so
//     outputs are bit-identical to the reference CPU aggregation.
//   * The per-client weight is wave-uniform: it is read with scalar loads
//     (s_load through the scalar cache, broadcast from SGPRs) — the CDNA way to
//     broadcast a uniform value, cheaper than an LDS round trip.
//   * k is unrolled U-deep: U rows of independent loads are issued before the
//     in-order adds consume them (the last B mod U rows too, under
//     wave-uniform guards), so every wave keeps several KiB in flight.
//   * HBM layout: the aggregator packs client rows into a COLUMN-BLOCKED slab
//     (a column block holds all K rows of its C columns contiguously), so each
//     block's workgroups stream one contiguous region.  Those loads go through
//     one buffer descriptor per workgroup with the row in an SGPR soffset:
//     buffer_load_dword{,x2,x4} v, v_off, s[rsrc], s_row offen nt.
//   * Client tensors the caller keeps in HBM ("borrowed" rows, a device table
//     of row pointers) are read where they lie; from 2^22 columns on a lane
//     there owns two pieces of 128 columns, so a wave reads 1 KiB of each row
//     per visit as two 512-byte loads (k_reduce_narrow<..., PC = 2>).
//   * A fused server step reads its operands (cloud / aux / momentum buffer)
//     with the first row batch, so no wave ends waiting on a dependent load.
//   * Layout / mapping / unroll / nt were chosen by measurement
//     (tools/sweep_reduce.py, tools/sweep_mapping.py, tools/ab_mapping.py,
//     profiles/).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// (see __graft_entry__.build()).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <initializer_list>
#include <type_traits>

#include "../../include/fedagg.h"

// The reference rounds every product and every sum separately; forbid the
// compiler from fusing them into an FMA anywhere in this translation unit.
#pragma clang fp contract(off)

namespace {

constexpr int kBlock = 256;  // 4 waves of 64 lanes
// Lanes per narrow-mapping workgroup: one wave.  A workgroup's share of the
// rows is then 1/4 of a 256-lane one, so the dispatcher balances the tail of
// the grid more finely: +1.4 % at 1000 x 25 M, +1.6 % at 1000 x 199,210, even
// at 1.09 M / 3.125 M (tools/sweep_variants.py, profiles/r01as/, r01at/;
// 512 / 1024 lanes were 0.5 / 2 % slower than 256).
constexpr int kNarrowBlock = 64;
// Tuned defaults (profiles/r01_*: K=1000 x P=25M sweep on MI355X).
constexpr int kDefaultUnroll = 4;
constexpr int kDefaultVptSel = 2;  // 2 float4 slots per lane
constexpr int kDefaultBsSel = 1;   // blocked layout: 256-lane workgroups
constexpr int kRowsUnroll = 4;     // row-pointer fused step (fedagg_reduce_step_rows_f32)
constexpr int kRowsVpt = 2;
// Default column mapping = narrow (tools/sweep_mapping.py, tools/ab_mapping.py,
// profiles/r01r/, r01t/, interleaved A/B on MI355X):
//  * P < 2^20: one column per lane, U = 8.  The f32x4-slot kernels cannot fill
//    256 CUs there (P = 199,210: 6.1 vs 1.3 TB/s at K = 1000);
//  * P >= 2^20: two columns per lane, U = 16 (U = 8 from 2^24 on), even with
//    or ahead of the tuned f32x4 kernels: +0.5..1.3 % at 1000 x 25 M, +3.8 %
//    at 1000 x 6.25 M, +3.8..5.7 % at 10,000 x 3.125 M (config 4's shard);
//  * P >= 2^24 with few rows per launch (B <= 64): four columns per lane,
//    U = 8 (a workgroup's fixed costs are spread over few rows there).  Under
//    one-wave workgroups two columns win again from about B = 100 (+2.7 % at
//    100 x 125 M, +3.5 % at 128 x 25 M, +5 % at 128 x 2^24; profiles/r01bo/).
constexpr int64_t kNarrowWideP = int64_t(1) << 20;
constexpr int64_t kNarrowLongP = int64_t(1) << 24;
constexpr int64_t kNarrowShortB = 64;

// Native clang vector (HIP's float4 is a struct and cannot feed the
// nontemporal builtin).
using f32x4 = float __attribute__((ext_vector_type(4)));
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x16 = float __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// Row addressing policies
// ---------------------------------------------------------------------------
struct RowsStrided {
  const float* X;
  int64_t ldx;
  __device__ __forceinline__ const char* row(int64_t k) const {
    return reinterpret_cast<const char*>(X + k * ldx);
  }
  template <bool NT>
  __device__ __forceinline__ f32x4 load4(int64_t k, uint32_t goff) const;
};

// Column-blocked slab: for column block b (C floats = one workgroup's span),
// rows 0..Kcap-1 are contiguous, so a workgroup streams one contiguous
// Kcap*C*4-byte region (TLB/DRAM-page friendly).  Element (k, p) lives at
// X[((p / C) * Kcap + k) * C + p % C].  row(k) is biased by -b*C so that the
// kernel's global slot offsets land inside block b's region.
struct RowsBlocked {
  const float* X;
  int64_t Kcap;
  int64_t C;
  __device__ __forceinline__ const char* row(int64_t k) const {
    return reinterpret_cast<const char*>(
        X + (static_cast<int64_t>(blockIdx.x) * (Kcap - 1) + k) * C);
  }
  template <bool NT>
  __device__ __forceinline__ f32x4 load4(int64_t k, uint32_t goff) const;
};

// Same layout, loaded with buffer instructions: the workgroup's region is one
// buffer descriptor (SGPRs), the row is an SGPR soffset (k * C * 4) and the
// lane's column is a 32-bit VGPR voffset, so every load is
//   buffer_load_dwordx4 v, v_off, s[rsrc], s_row offen [nt]
// and the unrolled loop needs one VGPR per column slot for addressing instead
// of a 64-bit VGPR pointer per in-flight load (134 -> ~90 VGPRs at U=4, VPT=4).
struct RowsBlockedBuf {
  const float* X;
  int64_t Kcap;
  int64_t C;
  __device__ __forceinline__ const char* row(int64_t k) const {
    return reinterpret_cast<const char*>(
        X + (static_cast<int64_t>(blockIdx.x) * (Kcap - 1) + k) * C);
  }
  template <bool NT>
  __device__ __forceinline__ f32x4 load4(int64_t k, uint32_t goff) const {
    const char* region = reinterpret_cast<const char*>(X + static_cast<int64_t>(blockIdx.x) * Kcap * C);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(region), static_cast<short>(0),
        static_cast<int>(static_cast<uint32_t>(Kcap * C * 4)), 0x00020000);
    const uint32_t voff = goff - static_cast<uint32_t>(blockIdx.x) * static_cast<uint32_t>(C * 4);
    const uint32_t soff = static_cast<uint32_t>(k) * static_cast<uint32_t>(C * 4);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(voff),
                                                          static_cast<int>(soff), NT ? 2 : 0);
    return __builtin_bit_cast(f32x4, v);
  }
};

// Row-pointer table loaded with buffer instructions: row k's base pointer is a
// wave-uniform scalar load from the table, turned into a buffer descriptor in
// SGPRs, and the lane's column stays a 32-bit VGPR voffset, so the unrolled
// loop holds no 64-bit VGPR address per in-flight load:
//   s_load_dwordx2 s[base], s[tab], k*8 ; buffer_load_dwordx4 v, v_off, s[rsrc], 0 offen
struct RowsTableBuf {
  const float* const* rows;
  uint32_t row_bytes;  // 4*P, clamped to the 32-bit field (table_row_bytes)
  __device__ __forceinline__ const char* row(int64_t k) const {
    return reinterpret_cast<const char*>(rows[k]);
  }
  template <bool NT>
  __device__ __forceinline__ f32x4 load4(int64_t k, uint32_t goff) const {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(rows[k]), static_cast<short>(0), static_cast<int>(row_bytes),
        0x00020000);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(goff), 0,
                                                          NT ? 2 : 0);
    return __builtin_bit_cast(f32x4, v);
  }
};

template <bool NT>
__device__ __forceinline__ f32x4 ld4(const char* base, uint32_t off) {
  const f32x4* p = reinterpret_cast<const f32x4*>(base + off);
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

template <bool NT>
__device__ __forceinline__ f32x4 RowsStrided::load4(int64_t k, uint32_t goff) const {
  return ld4<NT>(row(k), goff);
}
template <bool NT>
__device__ __forceinline__ f32x4 RowsBlocked::load4(int64_t k, uint32_t goff) const {
  return ld4<NT>(row(k), goff);
}
template <bool NT>
__device__ __forceinline__ float ld1(const char* base, uint32_t off) {
  const float* p = reinterpret_cast<const float*>(base + off);
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

// acc = fl32(acc + fl32(x * w)) — two roundings, as ATen CPU mul then add.
__device__ __forceinline__ float axpy_rn(float acc, float x, float w) {
  const float prod = x * w;
  return acc + prod;
}

__device__ __forceinline__ f32x4 axpy_rn4(f32x4 a, f32x4 x, float w) {
  a.x = axpy_rn(a.x, x.x, w);
  a.y = axpy_rn(a.y, x.y, w);
  a.z = axpy_rn(a.z, x.z, w);
  a.w = axpy_rn(a.w, x.w, w);
  return a;
}

__device__ __forceinline__ f32x4 div4(f32x4 a, float d) {
  // correctly rounded IEEE division (hipcc default
  // -fhip-fp32-correctly-rounded-divide-sqrt); NOT a * (1/d).
  a.x = a.x / d;
  a.y = a.y / d;
  a.z = a.z / d;
  a.w = a.w / d;
  return a;
}

// ---------------------------------------------------------------------------
// Server step: the algorithm's pseudo-gradient followed by the full
// torch.optim.SGD single-tensor update (torch/optim/sgd.py _single_tensor_sgd,
// the path torch takes for CPU params), with every ATen op's rounding:
//   d = maximize ? -g : g
//   d = fma(param, wd, d)                         grad.add(param, alpha=wd)
//   buf = first ? d : fma(d, 1-damp, fl(buf*m))   buf.mul_(m).add_(d, alpha=1-damp)
//   d = nesterov ? fma(buf, m, d) : buf           grad.add(buf, alpha=m)
//   param = fma(d, -lr, param)                    param.add_(d, alpha=-lr)
// ---------------------------------------------------------------------------
struct SgdArgs {
  float neg_lr, momentum, one_minus_damp, wd;
  int nesterov, maximize, first;
};

struct StepOut {
  float cloud, g, aux, buf;
};

// One column: a = average, c = cloud, x = aux (AdaBest avg_params / FedDyn h),
// b = momentum buffer.
template <int ALGO, bool MOM>
__device__ __forceinline__ StepOut step_math(float a, float c, float x, float b, float coef,
                                             const SgdArgs& sa) {
  StepOut o;
  float g;
  if constexpr (ALGO == FEDAGG_ALGO_FEDAVG) {
    g = c - a;  // fedavg.py:199
    o.aux = x;
  } else if constexpr (ALGO == FEDAGG_ALGO_ADABEST) {
    const float h = coef * (x - a);  // adabest.py:178-180
    const float nw = a - h;
    g = c - nw;
    o.aux = a;  // avg_params <- avg (adabest.py:188)
  } else {
    const float g1 = c - a;  // feddyn.py:176-184
    const float hn = x + coef * g1;
    const float nw = a - hn;
    g = c - nw;
    o.aux = hn;
  }
  o.g = g;
  float d = sa.maximize ? -g : g;
  if (sa.wd != 0.f) d = __builtin_fmaf(c, sa.wd, d);
  o.buf = b;
  if constexpr (MOM) {
    const float nb = sa.first ? d : __builtin_fmaf(d, sa.one_minus_damp, b * sa.momentum);
    o.buf = nb;
    d = sa.nesterov ? __builtin_fmaf(nb, sa.momentum, d) : nb;
  }
  o.cloud = __builtin_fmaf(d, sa.neg_lr, c);
  return o;
}

// ---------------------------------------------------------------------------
// Epilogues: what a kernel does with a finished column value (the average, or
// the raw sum).  `off` is the column's byte offset in a [P] vector.
// ---------------------------------------------------------------------------
// Epilogue operands, read with the first row batch (k_reduce_narrow).
template <class V>
struct EpiOps {
  V c, x, b;
};

struct EpiStore {  // plain reduce: store it
  float* out;
  template <class V>  // f32x4 / f32x2 columns at byte offset `off`
  __device__ __forceinline__ void vec(int64_t off, V a) const {
    *reinterpret_cast<V*>(reinterpret_cast<char*>(out) + off) = a;
  }
  template <class V>
  __device__ __forceinline__ EpiOps<V> load_ops(int64_t) const { return {}; }
  template <class V>
  __device__ __forceinline__ void pin(EpiOps<V>&) const {}
  template <class V>
  __device__ __forceinline__ void vec_with(int64_t off, V a, const EpiOps<V>&) const { vec(off, a); }
  __device__ __forceinline__ void one(int64_t col, float a) const { out[col] = a; }
};

struct StepPtrs {
  float* cloud;
  float* aux;
  float* avg_prev;
  float* buf;
  float* grad;
  float* avg_out;
  float coef;
  SgdArgs sa;
};

template <int ALGO, bool MOM>
struct EpiStep {  // server step on the average, in registers
  static constexpr int kAlgo = ALGO;
  static constexpr bool kMom = MOM;
  StepPtrs p;
  __device__ __forceinline__ void one(int64_t i, float a) const {
    const float x = (ALGO != FEDAGG_ALGO_FEDAVG) ? p.aux[i] : 0.f;
    const float b = MOM ? p.buf[i] : 0.f;
    const StepOut o = step_math<ALGO, MOM>(a, p.cloud[i], x, b, p.coef, p.sa);
    if (p.avg_out) p.avg_out[i] = a;
    if (p.grad) p.grad[i] = o.g;
    if constexpr (ALGO != FEDAGG_ALGO_FEDAVG) p.aux[i] = o.aux;
    if constexpr (ALGO == FEDAGG_ALGO_FEDDYN) {
      if (p.avg_prev) p.avg_prev[i] = a;
    }
    if constexpr (MOM) p.buf[i] = o.buf;
    p.cloud[i] = o.cloud;
  }
  template <class V>  // the step's operands of the columns at byte offset `off`
  __device__ __forceinline__ EpiOps<V> load_ops(int64_t off) const {
    auto at = [off](float* q) {
      return reinterpret_cast<const V*>(reinterpret_cast<const char*>(q) + off);
    };
    EpiOps<V> o{};
    o.c = *at(p.cloud);
    if constexpr (ALGO != FEDAGG_ALGO_FEDAVG) o.x = *at(p.aux);
    if constexpr (MOM) o.b = *at(p.buf);
    return o;
  }
  // keeps the compiler from sinking load_ops past the row loop: the values
  // must be in VGPRs here (one wait, while the first row batch is in flight)
  template <class V>
  __device__ __forceinline__ void pin(EpiOps<V>& o) const {
    asm volatile("" : "+v"(o.c));
    if constexpr (ALGO != FEDAGG_ALGO_FEDAVG) asm volatile("" : "+v"(o.x));
    if constexpr (MOM) asm volatile("" : "+v"(o.b));
  }
  template <class V>  // f32x4 / f32x2 columns at byte offset `off`
  __device__ __forceinline__ void vec(int64_t off, V a) const {
    vec_with(off, a, load_ops<V>(off));
  }
  template <class V>
  __device__ __forceinline__ void vec_with(int64_t off, V a, const EpiOps<V>& o) const {
    constexpr int N = sizeof(V) / sizeof(float);
    auto at = [off](float* q) {
      return reinterpret_cast<V*>(reinterpret_cast<char*>(q) + off);
    };
    const V c = o.c, x = o.x, b = o.b;
    V nc, g, nx, nb;
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const StepOut o = step_math<ALGO, MOM>(a[e], c[e], x[e], b[e], p.coef, p.sa);
      nc[e] = o.cloud;
      g[e] = o.g;
      nx[e] = o.aux;
      nb[e] = o.buf;
    }
    if (p.avg_out) *at(p.avg_out) = a;
    if (p.grad) *at(p.grad) = g;
    if constexpr (ALGO != FEDAGG_ALGO_FEDAVG) *at(p.aux) = nx;
    if constexpr (ALGO == FEDAGG_ALGO_FEDDYN) {
      if (p.avg_prev) *at(p.avg_prev) = a;
    }
    if constexpr (MOM) *at(p.buf) = nb;
    *at(p.cloud) = nc;
  }
};

// ---------------------------------------------------------------------------
// Exact-mode reduction, f32x4 slots.
//   slot s covers columns [4s, 4s+4).  Block b (BS lanes) owns slots
//   [b*BS*VPT, (b+1)*BS*VPT); lane t of the block owns s = base + j*BS + t
//   for j < VPT, so every wave-instruction touches 64 consecutive slots (1 KiB).
// ---------------------------------------------------------------------------
// Per-client weights: wave-uniform scalar loads.
struct WeightsScalar {
  const float* __restrict__ w;
  __device__ __forceinline__ float operator()(int64_t k) const { return w[k]; }
};

// Rows kb..ke-1 in order, U rows of loads in flight before the in-order adds.
template <int U, int VPT, bool NT, class Rows, class Wf>
__device__ __forceinline__ void accumulate_rows(const Rows& rows, const Wf& wf, int64_t kb,
                                                int64_t ke, const uint32_t* off, f32x4* a) {
  int64_t k = kb;
  for (; k + U <= ke; k += U) {
    f32x4 v[U][VPT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) v[u][j] = rows.template load4<NT>(k + u, off[j]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wk = wf(k + u);
#pragma unroll
      for (int j = 0; j < VPT; ++j) a[j] = axpy_rn4(a[j], v[u][j], wk);
    }
  }
  for (; k < ke; ++k) {
    const float wk = wf(k);
#pragma unroll
    for (int j = 0; j < VPT; ++j) a[j] = axpy_rn4(a[j], rows.template load4<NT>(k, off[j]), wk);
  }
}

template <int BS, int U, int VPT, bool NT, bool GUARD, class Rows, class Epi>
__device__ __forceinline__ void reduce_vec_body(const Rows& rows,
                                                const float* __restrict__ w,
                                                int64_t B, int64_t nvec,
                                                const float* acc_in, const Epi& epi,
                                                float W32, int flags) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (BS * VPT) + threadIdx.x;
  uint32_t off[VPT];
  bool ok[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    int64_t s = base + j * BS;
    ok[j] = GUARD ? (s < nvec) : true;
    if (GUARD && !ok[j]) s = nvec - 1;  // clamp: load something valid, store nothing
    off[j] = static_cast<uint32_t>(s) * 16u;
  }

  f32x4 a[VPT];
  if (flags & FEDAGG_INIT) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) a[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int j = 0; j < VPT; ++j)
      a[j] = ld4<false>(reinterpret_cast<const char*>(acc_in), off[j]);
  }

  // the per-client weight is wave-uniform: scalar loads (an LDS-staged
  // variant measured no better, DESIGN §3, and was removed)
  accumulate_rows<U, VPT, NT>(rows, WeightsScalar{w}, 0, B, off, a);

  if (flags & FEDAGG_FINALIZE) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) a[j] = div4(a[j], W32);
  }
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    if (ok[j]) epi.vec(off[j], a[j]);
  }
}

// Scalar columns [col0, col0 + ncols): the P % 4 tail of the f32x4 path.
template <bool NT, class Rows, class Epi>
__device__ __forceinline__ void reduce_scalar_cols(const Rows& rows,
                                                   const float* __restrict__ w,
                                                   int64_t B, int64_t col,
                                                   const float* acc_in, const Epi& epi,
                                                   float W32, int flags) {
  const uint32_t off = static_cast<uint32_t>(col) * 4u;
  float a = (flags & FEDAGG_INIT) ? 0.f : acc_in[col];
  for (int64_t k = 0; k < B; ++k) a = axpy_rn(a, ld1<NT>(rows.row(k), off), w[k]);
  if (flags & FEDAGG_FINALIZE) a = a / W32;
  epi.one(col, a);
}

template <int BS, int U, int VPT, bool NT, class Rows, class Epi = EpiStore>
__global__ __launch_bounds__(BS) void k_reduce_vec(Rows rows,
                                                       const float* __restrict__ w,
                                                       int64_t B, int64_t nvec,
                                                       int tail, const float* acc_in,
                                                       Epi epi, float W32,
                                                       int flags) {
  const int64_t block_start = static_cast<int64_t>(blockIdx.x) * (BS * VPT);
  const int64_t block_end = block_start + BS * VPT;
  if (block_end <= nvec) {
    reduce_vec_body<BS, U, VPT, NT, false>(rows, w, B, nvec, acc_in, epi, W32, flags);
  } else if (block_start < nvec) {
    reduce_vec_body<BS, U, VPT, NT, true>(rows, w, B, nvec, acc_in, epi, W32, flags);
  }
  // The last block also owns the (P % 4) scalar tail columns.
  if (blockIdx.x == gridDim.x - 1 && static_cast<int>(threadIdx.x) < tail)
    reduce_scalar_cols<NT>(rows, w, B, nvec * 4 + threadIdx.x, acc_in, epi, W32, flags);
}


// ---------------------------------------------------------------------------
// Narrow mapping for small P: VW (1 or 2) columns per lane instead of f32x4
// slots.  VW = 1 is also the path for rows that are not 16-byte aligned.    An in-order per-column sum has no parallelism but its columns, so
// at the reference's model sizes (SimpleMLP P = 199,210: 49,802 f32x4 slots =
// 778 waves, under one per SIMD) the wide kernel leaves most of the chip idle.
// One column per lane gives P lanes (3,113 waves there); U rows of dword loads
// stay in flight per lane.  Same per-element arithmetic and order.
// ---------------------------------------------------------------------------
using f32x2 = float __attribute__((ext_vector_type(2)));
using u32x2 = unsigned int __attribute__((ext_vector_type(2)));

template <int VW>
struct Cols {
  float v[VW];
};

template <int VW, bool NT>
__device__ __forceinline__ Cols<VW> buf_load_cols(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                                  uint32_t soff) {
  Cols<VW> o;
  if constexpr (VW == 1) {
    o.v[0] = __builtin_bit_cast(
        float, __builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(voff),
                                                    static_cast<int>(soff), NT ? 2 : 0));
  } else if constexpr (VW == 2) {
    const f32x2 t = __builtin_bit_cast(
        f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, static_cast<int>(voff),
                                                    static_cast<int>(soff), NT ? 2 : 0));
    o.v[0] = t.x;
    o.v[1] = t.y;
  } else {
    const f32x4 t = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(voff),
                                                     static_cast<int>(soff), NT ? 2 : 0));
#pragma unroll
    for (int e = 0; e < 4; ++e) o.v[e] = t[e];
  }
  return o;
}

// Row-address prefetch for k_reduce_narrow's main loop.  Policies whose row
// address is arithmetic have nothing to fetch; the pointer-table policy loads
// the next batch's U row pointers while the current batch's rows stream.
struct NoRowPrefetch {};
#define FEDAGG_NO_ROW_PREFETCH                                                              \
  template <int U>                                                                          \
  __device__ __forceinline__ NoRowPrefetch prefetch(int64_t) const {                        \
    return {};                                                                              \
  }                                                                                         \
  template <int VW, bool NT, int U>                                                         \
  __device__ __forceinline__ Cols<VW> load_at(const NoRowPrefetch&, int64_t k, int u,       \
                                              uint32_t voff) const {                        \
    return load<VW, NT>(k + u, voff);                                                       \
  }

// Column-blocked slab: the workgroup's 256*VW columns lie in one column block
// b (C is a multiple of 256*VW); its region is one buffer descriptor, the row
// an SGPR soffset, the lane's column-in-block a VGPR voffset.
struct NarrowBlocked {
  const float* X;
  int64_t Kcap;
  int64_t C;
  template <int VW>
  __device__ __forceinline__ uint32_t lane_off(int64_t c) const {
    return static_cast<uint32_t>(c & (C - 1)) * 4u;
  }
  // SPAN: columns one workgroup covers (all inside one block)
  template <int VW, bool NT, int SPAN = kNarrowBlock * VW>
  __device__ __forceinline__ Cols<VW> load(int64_t k, uint32_t voff) const {
    const int64_t b = (static_cast<int64_t>(blockIdx.x) * SPAN) >> __builtin_ctzll(C);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(X + b * Kcap * C), static_cast<short>(0),
        static_cast<int>(static_cast<uint32_t>(Kcap * C * 4)), 0x00020000);
    return buf_load_cols<VW, NT>(r, voff, static_cast<uint32_t>(k) * static_cast<uint32_t>(C * 4));
  }  FEDAGG_NO_ROW_PREFETCH
};

// Row-pointer table: one descriptor per row (wave-uniform scalar load).
struct NarrowTable {
  const float* const* rows;
  uint32_t row_bytes;
  template <int VW>
  __device__ __forceinline__ uint32_t lane_off(int64_t c) const {
    return static_cast<uint32_t>(c) * 4u;
  }
  template <int VW, bool NT, int SPAN = kNarrowBlock * VW>
  __device__ __forceinline__ Cols<VW> load(int64_t k, uint32_t voff) const {
    return load_row<VW, NT>(rows[k], voff);
  }
  template <int U>
  struct Batch {
    const float* p[U];
  };
  // the U row pointers of rows k .. k+U-1 (scalar loads, in SGPRs)
  template <int U>
  __device__ __forceinline__ Batch<U> prefetch(int64_t k) const {
    Batch<U> b;
#pragma unroll
    for (int u = 0; u < U; ++u) b.p[u] = rows[k + u];
    return b;
  }
  template <int VW, bool NT, int U>
  __device__ __forceinline__ Cols<VW> load_at(const Batch<U>& b, int64_t, int u,
                                              uint32_t voff) const {
    return load_row<VW, NT>(b.p[u], voff);
  }
  template <int VW, bool NT>
  __device__ __forceinline__ Cols<VW> load_row(const float* row, uint32_t voff) const {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(row), static_cast<short>(0), static_cast<int>(row_bytes), 0x00020000);
    return buf_load_cols<VW, NT>(r, voff, 0u);
  }
};

// Row-pointer table with flat loads, for rows a descriptor cannot cover: its
// range check is on the access's end, so a row of exactly 2^32 bytes
// (P = 2^30, the largest P accepted) would read its last columns as zero.
struct NarrowTableFlat {
  const float* const* rows;
  template <int VW>
  __device__ __forceinline__ uint32_t lane_off(int64_t c) const {
    return static_cast<uint32_t>(c) * 4u;
  }
  template <int VW, bool NT, int SPAN = kNarrowBlock * VW>
  __device__ __forceinline__ Cols<VW> load(int64_t k, uint32_t voff) const {
    static_assert(VW == 1, "flat table rows: one column per lane");
    Cols<VW> o;
    o.v[0] = ld1<NT>(reinterpret_cast<const char*>(rows[k]), voff);
    return o;
  }  FEDAGG_NO_ROW_PREFETCH
};

// A row's byte length fits one buffer descriptor (num_records is 32 bits and
// checked against the access's end).
inline bool row_fits_descriptor(int64_t P) { return P * 4 <= int64_t(0xFFFFFFFF); }

// Row-major [B, ldx] slab (may exceed a descriptor's 4 GiB range): flat loads.
struct NarrowStrided {
  const float* X;
  int64_t ldx;
  template <int VW>
  __device__ __forceinline__ uint32_t lane_off(int64_t c) const {
    return static_cast<uint32_t>(c) * 4u;
  }
  template <int VW, bool NT, int SPAN = kNarrowBlock * VW>
  __device__ __forceinline__ Cols<VW> load(int64_t k, uint32_t voff) const {
    const char* p = reinterpret_cast<const char*>(X + k * ldx) + voff;
    Cols<VW> o;
    if constexpr (VW == 1) {
      o.v[0] = ld1<NT>(p, 0);
    } else if constexpr (VW == 2) {
      const f32x2* q = reinterpret_cast<const f32x2*>(p);
      const f32x2 t = NT ? __builtin_nontemporal_load(q) : *q;
      o.v[0] = t.x;
      o.v[1] = t.y;
    } else {
      const f32x4 t = ld4<NT>(p, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) o.v[e] = t[e];
    }
    return o;
  }  FEDAGG_NO_ROW_PREFETCH
};

template <int VW> struct EpiVec { using type = f32x4; };
template <> struct EpiVec<2> { using type = f32x2; };

// PC pieces per lane: lane t owns columns c0 + j*64*VW .. +VW-1 for j < PC, so
// one wave reads PC * 64 * VW * 4 contiguous bytes of each row per visit, as PC
// separate VW-wide loads (PC = 2 for borrowed rows, see the dispatch; the
// column-blocked slab keeps PC = 1, its workgroup span must stay in a block).
template <int U, int VW, bool NT, class NR, class Epi, int PC = 1>
__global__ __launch_bounds__(kNarrowBlock) void k_reduce_narrow(NR rows, const float* __restrict__ w,
                                                          int64_t B, int64_t P,
                                                          const float* acc_in, Epi epi,
                                                          float W32, int flags) {
  constexpr int64_t kPiece = int64_t(kNarrowBlock) * VW;  // columns of one piece
  const int64_t cb = static_cast<int64_t>(blockIdx.x) * kPiece * PC + threadIdx.x * VW;
  int64_t c0[PC], c[PC];
  bool ok[PC];
  uint32_t voff[PC];
  float a[PC][VW];
#pragma unroll
  for (int j = 0; j < PC; ++j) {
    c0[j] = cb + j * kPiece;
    ok[j] = c0[j] < P;
    c[j] = ok[j] ? c0[j] : P - VW;  // clamp: load something valid, store nothing
    voff[j] = rows.template lane_off<VW>(c[j]);
#pragma unroll
    for (int e = 0; e < VW; ++e) a[j][e] = (flags & FEDAGG_INIT) ? 0.f : acc_in[c[j] + e];
  }
  int64_t k = 0;
  // The step's operands (cloud / aux / momentum buffer) are read with the
  // first row batch, not after the last one: a wave that ends in a dependent
  // load keeps its slot from streaming rows for a memory latency (+0.5 % at
  // 1000 x 25 M, +0.5..1.1 % at 1..8 M columns; profiles/r01bw/).
  using EV = typename EpiVec<VW>::type;
  EpiOps<EV> pre[PC]{};
  if constexpr (VW >= 2) {
#pragma unroll
    for (int j = 0; j < PC; ++j) pre[j] = epi.template load_ops<EV>(c[j] * 4);
  }
  bool pinned = false;
  // row addresses of the next batch are fetched while this batch streams
  // (clamped to the last full batch, so the table is never over-read)
  decltype(rows.template prefetch<U>(0)) next{};
  if (U <= B) next = rows.template prefetch<U>(0);
  for (; k + U <= B; k += U) {
    const auto cur = next;
    Cols<VW> v[U][PC];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < PC; ++j) v[u][j] = rows.template load_at<VW, NT, U>(cur, k, u, voff[j]);
    next = rows.template prefetch<U>(k + 2 * U <= B ? k + U : k);
    if constexpr (VW >= 2) {
      if (!pinned) {
#pragma unroll
        for (int j = 0; j < PC; ++j) epi.pin(pre[j]);
        pinned = true;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wk = w[k + u];
#pragma unroll
      for (int j = 0; j < PC; ++j)
#pragma unroll
        for (int e = 0; e < VW; ++e) a[j][e] = axpy_rn(a[j][e], v[u][j].v[e], wk);
    }
  }
  if (k < B) {
    // the last B % U rows: one load per lane per row, so a plain tail loop
    // would wait out a full memory latency per row (what small-K rounds are
    // made of); issue them all before the in-order adds, under wave-uniform
    // guards
    const int64_t rem = B - k;
    Cols<VW> v[U - 1][PC];
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (u < rem) {
#pragma unroll
        for (int j = 0; j < PC; ++j) v[u][j] = rows.template load<VW, NT>(k + u, voff[j]);
      }
#pragma unroll
    for (int u = 0; u < U - 1; ++u) {
      if (u < rem) {
        const float wk = w[k + u];
#pragma unroll
        for (int j = 0; j < PC; ++j)
#pragma unroll
          for (int e = 0; e < VW; ++e) a[j][e] = axpy_rn(a[j][e], v[u][j].v[e], wk);
      }
    }
  }
  if (flags & FEDAGG_FINALIZE) {
#pragma unroll
    for (int j = 0; j < PC; ++j)
#pragma unroll
      for (int e = 0; e < VW; ++e) a[j][e] = a[j][e] / W32;
  }
#pragma unroll
  for (int j = 0; j < PC; ++j) {
    if (ok[j]) {
      if constexpr (VW == 4) {
        epi.vec_with(c0[j] * 4, f32x4{a[j][0], a[j][1], a[j][2], a[j][3]}, pre[j]);
      } else if constexpr (VW == 2) {
        epi.vec_with(c0[j] * 4, f32x2{a[j][0], a[j][1]}, pre[j]);
      } else {
        epi.one(c0[j], a[j][0]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Fast (reordered) mode, FEDAGG_FAST: split-K for few columns and many rows.
// Below ~64 columns per SIMD even one column per lane cannot fill the chip
// (a 7,850-parameter logistic regression is 123 waves), so the K rows of a
// 64-column tile are split over the S waves of a workgroup:
//   * wave s takes rows k0 + s*U .. k0 + s*U + U-1 of every S*U-row step;
//     lane l owns column tile*64 + l (256 B per wave-instruction);
//   * the per-client weights of a 4096-row tile are staged once in LDS by the
//     whole workgroup and read back as wave-uniform (broadcast) ds_reads;
//   * each wave keeps a running fmaf partial sum; the S partials are combined
//     through LDS by wave 0 in a fixed order (s = 0..S-1, then acc_in), so the
//     result is deterministic run to run but NOT the reference's summation
//     order: parity is normwise, like the client-sharded
//     all-reduce.
// ---------------------------------------------------------------------------
constexpr int kSplitWeights = 4096;

template <int S, int U, bool NT, class NR, class Epi>
__global__ __launch_bounds__(64 * S) void k_reduce_splitk(NR rows, const float* __restrict__ w,
                                                          int64_t B, int64_t P,
                                                          const float* acc_in, Epi epi,
                                                          float W32, int flags) {
  __shared__ float wsh[kSplitWeights];
  __shared__ float part[S][64];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  const bool ok = c0 < P;
  const int64_t c = ok ? c0 : P - 1;
  const uint32_t voff = rows.template lane_off<1>(c);
  float a = 0.f;
  for (int64_t t0 = 0; t0 < B; t0 += kSplitWeights) {
    const int64_t n = (B - t0) < kSplitWeights ? (B - t0) : kSplitWeights;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < n; i += 64 * S) wsh[i] = w[t0 + i];
    __syncthreads();
    int64_t k = wv * U;  // tile-relative row of this wave's first load
    for (; k + U <= n; k += S * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = rows.template load<1, NT, 64>(t0 + k + u, voff).v[0];
#pragma unroll
      for (int u = 0; u < U; ++u) a = __builtin_fmaf(v[u], wsh[k + u], a);
    }
    if (k < n) {  // this wave's last, partial step of the tile
      const int64_t rem = n - k;
      float v[U - 1];
#pragma unroll
      for (int u = 0; u < U - 1; ++u)
        if (u < rem) v[u] = rows.template load<1, NT, 64>(t0 + k + u, voff).v[0];
#pragma unroll
      for (int u = 0; u < U - 1; ++u)
        if (u < rem) a = __builtin_fmaf(v[u], wsh[k + u], a);
    }
  }
  part[wv][lane] = a;
  __syncthreads();
  if (wv == 0) {
    float t = part[0][lane];
#pragma unroll
    for (int q = 1; q < S; ++q) t = t + part[q][lane];
    if (!(flags & FEDAGG_INIT)) t = acc_in[c] + t;
    if (flags & FEDAGG_FINALIZE) t = t / W32;
    if (ok) epi.one(c0, t);
  }
}

// ---------------------------------------------------------------------------
// Elementwise epilogues (grid-stride, f32x4 body + scalar tail).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_finalize(const float* acc, float W32,
                                                     int64_t P, float* out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t nvec = P / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < nvec; i += stride) {
    f32x4 a = reinterpret_cast<const f32x4*>(acc)[i];
    reinterpret_cast<f32x4*>(out)[i] = div4(a, W32);
  }
  if (blockIdx.x == 0 && static_cast<int64_t>(threadIdx.x) < P - nvec * 4) {
    const int64_t c = nvec * 4 + threadIdx.x;
    out[c] = acc[c] / W32;
  }
}

// f64 true division (the fp64 keys of the dtype-generic aggregator); two
// doubles per lane per iteration, 16-B loads
__global__ __launch_bounds__(kBlock) void k_finalize_f64(const double* acc, double W,
                                                         int64_t P, double* out) {
  using f64x2 = double __attribute__((ext_vector_type(2)));
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t nvec = P / 2;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < nvec; i += stride) {
    f64x2 a = reinterpret_cast<const f64x2*>(acc)[i];
    a.x = a.x / W;
    a.y = a.y / W;
    reinterpret_cast<f64x2*>(out)[i] = a;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (P & 1)) out[P - 1] = acc[P - 1] / W;
}

// torch CPU SGD.step = param.add_(grad, alpha=-lr) = fma(-lr, g, param)
__device__ __forceinline__ float sgd_rn(float c, float g, float neg_lr) {
  return __builtin_fmaf(neg_lr, g, c);
}

__device__ __forceinline__ void fedavg_elem(const float* avg, float neg_lr, float* cloud,
                                            float* grad_out, int64_t i) {
  const float c = cloud[i];
  const float g = c - avg[i];
  if (grad_out) grad_out[i] = g;
  cloud[i] = sgd_rn(c, g, neg_lr);
}

__global__ __launch_bounds__(kBlock) void k_fedavg_sgd(const float* __restrict__ avg,
                                                       float neg_lr,
                                                       float* __restrict__ cloud,
                                                       float* __restrict__ grad_out,
                                                       int64_t P) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t nvec = P / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < nvec; i += stride) {
    const f32x4 a = reinterpret_cast<const f32x4*>(avg)[i];
    f32x4 c = reinterpret_cast<f32x4*>(cloud)[i];
    f32x4 g;
    g.x = c.x - a.x; g.y = c.y - a.y; g.z = c.z - a.z; g.w = c.w - a.w;
    if (grad_out) reinterpret_cast<f32x4*>(grad_out)[i] = g;
    c.x = sgd_rn(c.x, g.x, neg_lr); c.y = sgd_rn(c.y, g.y, neg_lr);
    c.z = sgd_rn(c.z, g.z, neg_lr); c.w = sgd_rn(c.w, g.w, neg_lr);
    reinterpret_cast<f32x4*>(cloud)[i] = c;
  }
  if (blockIdx.x == 0 && static_cast<int64_t>(threadIdx.x) < P - nvec * 4)
    fedavg_elem(avg, neg_lr, cloud, grad_out, nvec * 4 + threadIdx.x);
}

__device__ __forceinline__ void adabest_elem(const float* avg, float beta, float neg_lr,
                                             float* cloud, float* avg_prev, float* grad_out,
                                             int64_t i) {
  const float a = avg[i];
  const float h = beta * (avg_prev[i] - a);
  const float nw = a - h;
  const float c = cloud[i];
  const float g = c - nw;
  if (grad_out) grad_out[i] = g;
  cloud[i] = sgd_rn(c, g, neg_lr);
  avg_prev[i] = a;
}

__global__ __launch_bounds__(kBlock) void k_adabest_sgd(const float* __restrict__ avg,
                                                        float beta, float neg_lr,
                                                        float* __restrict__ cloud,
                                                        float* __restrict__ avg_prev,
                                                        float* __restrict__ grad_out,
                                                        int64_t P) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < P; i += stride)
    adabest_elem(avg, beta, neg_lr, cloud, avg_prev, grad_out, i);
}

// D2D pack of one client vector into row r of a column-blocked slab: a
// streaming copy in tiles of kPackU * 1024 columns per workgroup, kPackU
// 16-B non-temporal loads in flight per lane before its 16-B non-temporal
// stores (both coalesced inside a column block; C is a multiple of 4).  The
// DMA engines are slower than the CUs for HBM->HBM copies.
constexpr int kPackU = 4;

__global__ __launch_bounds__(kBlock) void k_pack_row(const float* __restrict__ src,
                                                     int64_t P, float* __restrict__ Xb,
                                                     int64_t Kcap, int64_t C, int64_t r) {
  constexpr int64_t kTile = int64_t(kBlock) * 4 * kPackU;
  const int64_t nvec = P / 4;
  const int64_t ntiles = (P + kTile - 1) / kTile;
  const int64_t cvec = C / 4;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    f32x4 v[kPackU];
#pragma unroll
    for (int u = 0; u < kPackU; ++u) {
      const int64_t i = t * (kTile / 4) + int64_t(u) * kBlock + threadIdx.x;
      if (i < nvec) v[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src) + i);
    }
#pragma unroll
    for (int u = 0; u < kPackU; ++u) {
      const int64_t i = t * (kTile / 4) + int64_t(u) * kBlock + threadIdx.x;
      if (i < nvec) {
        const int64_t b = i / cvec;
        __builtin_nontemporal_store(v[u], reinterpret_cast<f32x4*>(Xb + (b * Kcap + r) * C) +
                                              (i - b * cvec));
      }
    }
  }
  if (blockIdx.x == 0 && static_cast<int64_t>(threadIdx.x) < P - nvec * 4) {
    const int64_t p = nvec * 4 + threadIdx.x;
    Xb[((p / C) * Kcap + r) * C + p % C] = src[p];
  }
}

inline int pack_grid(int64_t P) {
  const int64_t tiles = (P + int64_t(kBlock) * 4 * kPackU - 1) / (int64_t(kBlock) * 4 * kPackU);
  return static_cast<int>(tiles < 1 ? 1 : tiles < 8192 ? tiles : 8192);
}

// vectorize_module straight into a slab row: the concatenation of a model's
// parameter tensors (segments: {src, first column, length}, sorted, tiling
// [0, P)) written to row r of a column-blocked slab in one launch, in place of
// torch.cat + clone + pack (fedsim/utils/convert_parameters.py:78-94).
//
// A workgroup owns a tile of kPackU * 1024 consecutive columns; each lane owns
// kPackU quads of 4 columns (one 16-B non-temporal store each: C is a
// multiple of 4, so a quad never straddles a column block).  The tile's first
// segment is found once by binary search over the short, cache-resident
// table; lanes walk forward from it.  All of a lane's loads are issued before
// its stores.  A quad inside one segment loads 16 B when its source is 16-B
// aligned (a model whose parameters are views of one vector: one segment),
// else four 4-B loads; a quad across a segment boundary gathers per column.

__device__ __forceinline__ int64_t pack_seg_of(const int64_t* __restrict__ segs, int64_t nseg,
                                               int64_t p) {
  int64_t lo = 0, hi = nseg - 1;  // last segment whose first column <= p
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (segs[3 * mid + 1] <= p) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kBlock) void k_pack_segments(const int64_t* __restrict__ segs,
                                                          int64_t nseg, int64_t P,
                                                          float* __restrict__ Xb, int64_t Kcap,
                                                          int64_t C, int64_t r) {
  constexpr int64_t kTile = int64_t(kBlock) * 4 * kPackU;
  const int64_t ntiles = (P + kTile - 1) / kTile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t t0 = t * kTile;
    int64_t seg = pack_seg_of(segs, nseg, t0);
    f32x4 v[kPackU];
    int64_t pq[kPackU];
#pragma unroll
    for (int u = 0; u < kPackU; ++u) {
      const int64_t p = t0 + (int64_t(u) * kBlock + threadIdx.x) * 4;
      pq[u] = p;
      v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p >= P) continue;
      while (seg + 1 < nseg && segs[3 * (seg + 1) + 1] <= p) ++seg;
      const int64_t off = segs[3 * seg + 1];
      const int64_t end = off + segs[3 * seg + 2];
      const float* s = reinterpret_cast<const float*>(segs[3 * seg]) + (p - off);
      if (p + 4 <= end) {
        if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) {
          v[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s));
        } else {
          v[u] = f32x4{s[0], s[1], s[2], s[3]};
        }
      } else {  // the quad crosses a segment boundary, or P
        int64_t sg = seg;
        for (int j = 0; j < 4 && p + j < P; ++j) {
          while (sg + 1 < nseg && segs[3 * (sg + 1) + 1] <= p + j) ++sg;
          const int64_t o = segs[3 * sg + 1];
          if (p + j < o + segs[3 * sg + 2])  // a table that does not tile [0, P)
            v[u][j] = reinterpret_cast<const float*>(segs[3 * sg])[p + j - o];  // leaves 0
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kPackU; ++u) {
      const int64_t p = pq[u];
      if (p >= P) continue;
      float* dst = Xb + ((p / C) * Kcap + r) * C + p % C;
      if (p + 4 <= P) {
        __builtin_nontemporal_store(v[u], reinterpret_cast<f32x4*>(dst));
      } else {
        for (int j = 0; j < 4 && p + j < P; ++j) dst[j] = v[u][j];
      }
    }
  }
}

// Row r of a column-blocked slab back to a contiguous vector (a slab row
// handed out by vectorize_module, read as an ordinary tensor).
__global__ __launch_bounds__(kBlock) void k_unpack_row(const float* __restrict__ Xb,
                                                       int64_t Kcap, int64_t C, int64_t r,
                                                       int64_t P, float* __restrict__ dst) {
  const int64_t nvec = P / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t cvec = C / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < nvec; i += stride) {
    const int64_t b = i / cvec;
    const int64_t c = i - b * cvec;
    reinterpret_cast<f32x4*>(dst)[i] = reinterpret_cast<const f32x4*>(Xb + (b * Kcap + r) * C)[c];
  }
  if (blockIdx.x == 0 && static_cast<int64_t>(threadIdx.x) < P - nvec * 4) {
    const int64_t p = nvec * 4 + threadIdx.x;
    dst[p] = Xb[((p / C) * Kcap + r) * C + p % C];
  }
}

// FedDyn (feddyn.py:169-194): h += ratio * (cloud - avg); new = avg - h;
// cloud <- fma(-lr, cloud - new, cloud); avg_prev <- avg.
__global__ __launch_bounds__(kBlock) void k_feddyn_sgd(const float* __restrict__ avg,
                                                       float ratio, float neg_lr,
                                                       float* __restrict__ cloud,
                                                       float* __restrict__ h,
                                                       float* __restrict__ avg_prev,
                                                       float* __restrict__ grad_out,
                                                       int64_t P) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < P; i += stride) {
    const float a = avg[i];
    const float c = cloud[i];
    const float g1 = c - a;
    const float t = ratio * g1;
    const float hn = h[i] + t;
    const float nw = a - hn;
    const float g = c - nw;
    if (grad_out) grad_out[i] = g;
    cloud[i] = sgd_rn(c, g, neg_lr);
    h[i] = hn;
    if (avg_prev) avg_prev[i] = a;
  }
}

// ---------------------------------------------------------------------------
// General server step over a stored average (fedagg_server_step_f32): the
// EpiStep epilogue applied to avg[], f32x4 when every operand is 16-B aligned.
// ---------------------------------------------------------------------------
template <int ALGO, bool MOM, bool VEC>
__global__ __launch_bounds__(kBlock) void k_server_step(const float* __restrict__ avg,
                                                        EpiStep<ALGO, MOM> epi, int64_t P) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if constexpr (VEC) {
    const int64_t nvec = P / 4;
    for (int64_t i = t0; i < nvec; i += stride)
      epi.vec(i * 16, reinterpret_cast<const f32x4*>(avg)[i]);
    if (blockIdx.x == 0 && static_cast<int64_t>(threadIdx.x) < P - nvec * 4) {
      const int64_t c = nvec * 4 + threadIdx.x;
      epi.one(c, avg[c]);
    }
  } else {
    for (int64_t i = t0; i < P; i += stride) epi.one(i, avg[i]);
  }
}

// ---------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int elementwise_grid(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 256 * 8) g = 256 * 8;  // 8 blocks per CU, grid-stride the rest
  return static_cast<int>(g);
}

template <int BS, int U, int VPT, bool NT, class Rows, class Epi = EpiStore>
hipError_t launch_vec(const Rows& rows, const float* w, int64_t B, int64_t P,
                      const float* acc_in, const Epi& epi, float W32, int flags,
                      hipStream_t s) {
  const int64_t nvec = P / 4;
  const int tail = static_cast<int>(P - nvec * 4);
  // one workgroup per BS*VPT float4 slots; the scalar tail belongs to the
  // workgroup whose column span contains it (matters for RowsBlocked)
  int64_t grid = (nvec + (tail > 0 ? 1 : 0) + BS * VPT - 1) / (BS * VPT);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((k_reduce_vec<BS, U, VPT, NT, Rows, Epi>),
                     dim3(static_cast<unsigned>(grid)), dim3(BS), 0, s, rows, w, B, nvec, tail,
                     acc_in, epi, W32, flags);
  return hipGetLastError();
}

template <int BS, int VPT, bool NT, class Rows>
hipError_t dispatch_unroll(int unroll_sel, const Rows& rows, const float* w, int64_t B,
                           int64_t P, const float* acc_in, float* out, float W32,
                           int flags, hipStream_t s) {
  const EpiStore st{out};
  switch (unroll_sel) {
    case 1: return launch_vec<BS, 4, VPT, NT>(rows, w, B, P, acc_in, st, W32, flags, s);
    case 2: return launch_vec<BS, 8, VPT, NT>(rows, w, B, P, acc_in, st, W32, flags, s);
    case 3: return launch_vec<BS, 16, VPT, NT>(rows, w, B, P, acc_in, st, W32, flags, s);
    case 4: return launch_vec<BS, 2, VPT, NT>(rows, w, B, P, acc_in, st, W32, flags, s);
    case 0:
    default:
      return launch_vec<BS, kDefaultUnroll, VPT, NT>(rows, w, B, P, acc_in, st, W32, flags, s);
  }
}

template <int BS, int VPT, class Rows>
hipError_t dispatch_nt(const Rows& rows, const float* w, int64_t B, int64_t P,
                       const float* acc_in, float* out, float W32, int flags, hipStream_t s) {
  const int unroll_sel = (flags & FEDAGG_UNROLL_MASK) >> FEDAGG_UNROLL_SHIFT;
  return (flags & FEDAGG_NT)
             ? dispatch_unroll<BS, VPT, true>(unroll_sel, rows, w, B, P, acc_in, out, W32, flags, s)
             : dispatch_unroll<BS, VPT, false>(unroll_sel, rows, w, B, P, acc_in, out, W32, flags,
                                               s);
}

template <class Rows>
hipError_t dispatch_reduce(const Rows& rows, const float* w, int64_t B, int64_t P,
                           const float* acc_in, float* out, float W32, int flags, hipStream_t s) {
  const int vpt_sel = (flags & FEDAGG_VPT_MASK) >> FEDAGG_VPT_SHIFT;
  switch (vpt_sel == 0 ? kDefaultVptSel : vpt_sel) {
    case 1: return dispatch_nt<kBlock, 1>(rows, w, B, P, acc_in, out, W32, flags, s);
    case 3: return dispatch_nt<kBlock, 4>(rows, w, B, P, acc_in, out, W32, flags, s);
    case 2:
    default: return dispatch_nt<kBlock, 2>(rows, w, B, P, acc_in, out, W32, flags, s);
  }
}

// The column block is one workgroup's span: C = BS lanes * VPT slots * 4.
template <class Rows>
hipError_t dispatch_blocked(const Rows& rows, int64_t C, int bs_sel, const float* w, int64_t B,
                            int64_t P, const float* acc_in, float* out, float W32, int flags,
                            hipStream_t s) {
  if (C == 1024) return dispatch_nt<256, 1>(rows, w, B, P, acc_in, out, W32, flags, s);
  if (C == 2048)
    return bs_sel >= 2 ? dispatch_nt<512, 1>(rows, w, B, P, acc_in, out, W32, flags, s)
                       : dispatch_nt<256, 2>(rows, w, B, P, acc_in, out, W32, flags, s);
  if (C == 4096)
    return bs_sel == 3   ? dispatch_nt<1024, 1>(rows, w, B, P, acc_in, out, W32, flags, s)
           : bs_sel == 2 ? dispatch_nt<512, 2>(rows, w, B, P, acc_in, out, W32, flags, s)
                         : dispatch_nt<256, 4>(rows, w, B, P, acc_in, out, W32, flags, s);
  return hipErrorInvalidValue;
}

// num_records of a row's buffer descriptor: 4*P bytes (rows that do not fit,
// P = 2^30, take NarrowTableFlat; the clamp only keeps the value defined).
uint32_t table_row_bytes(int64_t P) {
  const int64_t b = P * 4;
  return b >= (int64_t(1) << 32) ? 0xFFFFFFFFu : static_cast<uint32_t>(b);
}

int check_reduce_args(const float* w, int64_t B, int64_t P, const float* acc_in,
                      const float* out, int flags) {
  if (B < 0 || P < 0) return FEDAGG_EINVAL;
  if (P > (int64_t(1) << 30)) return FEDAGG_EINVAL;  // 32-bit per-row byte offsets
  if (P == 0) return 0;
  if (!out) return FEDAGG_EINVAL;
  if (B > 0 && !w) return FEDAGG_EINVAL;
  if (!(flags & FEDAGG_INIT) && !acc_in) return FEDAGG_EINVAL;
  if (flags & ~(FEDAGG_INIT | FEDAGG_FINALIZE | FEDAGG_NT | FEDAGG_SCALAR | FEDAGG_UNROLL_MASK |
                FEDAGG_VPT_MASK | FEDAGG_BS_MASK | FEDAGG_MAP_MASK | FEDAGG_FAST))
    return FEDAGG_EINVAL;
  if (((flags & FEDAGG_MAP_MASK) >> FEDAGG_MAP_SHIFT) > 4) return FEDAGG_EINVAL;
  return 0;
}

// Columns per lane of the narrow mapping for this call, or 0 for the wide
// (f32x4-slot) kernels.  `vw_ok` says whether 2 columns per lane are possible
// (P even, 8-byte aligned operands).
int narrow_vw(int flags, int64_t P, int64_t B, int max_vw) {
  const int m = (flags & FEDAGG_MAP_MASK) >> FEDAGG_MAP_SHIFT;
  int vw;
  if (m == 1) return 0;
  if (m == 2) vw = 1;
  else if (m == 3) vw = 2;
  else if (m == 4) vw = 4;
  else if (P < kNarrowWideP) vw = 1;
  else vw = (P >= kNarrowLongP && B <= kNarrowShortB) ? 4 : 2;
  while (vw > max_vw) vw /= 2;
  return vw;
}

// The widest columns-per-lane (1 / 2 / 4) that P and the operands' alignment
// allow.
int max_cols_per_lane(int64_t P, std::initializer_list<const void*> ptrs) {
  int v = (P % 4 == 0) ? 4 : (P % 2 == 0) ? 2 : 1;
  for (const void* q : ptrs) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(q);
    if (v == 4 && (a & 15u)) v = 2;
    if (v == 2 && (a & 7u)) v = 1;
  }
  return v;
}

// Borrowed rows (pointer table) with two columns per lane read two pieces per
// lane from P >= kRowsPiecesP on, with at most kRowsPiecesU rows in flight
// (profiles/r01cf/).
// (Round 5: 4 / 8 / 16 pieces with 2..8 rows in flight measured no faster at
// 1000 x 25 M / 12.5 M, profiles/r05p/.)
constexpr int kRowsPieces = 2;
constexpr int kRowsPiecesU = 8;
constexpr int64_t kRowsPiecesP = int64_t(1) << 22;

template <int U, int VW, bool NT, class NR, class Epi>
hipError_t launch_narrow_t(const NR& rows, const float* w, int64_t B, int64_t P,
                           const float* acc_in, const Epi& epi, float W32, int flags,
                           hipStream_t s) {
  if constexpr (std::is_same_v<NR, NarrowTable> && VW == 2 && kRowsPieces > 1) {
    if (P >= kRowsPiecesP) {
      constexpr int UP = U < kRowsPiecesU ? U : kRowsPiecesU;
      constexpr int64_t span = int64_t(kNarrowBlock) * VW * kRowsPieces;
      const int64_t g = (P + span - 1) / span;
      hipLaunchKernelGGL((k_reduce_narrow<UP, VW, NT, NR, Epi, kRowsPieces>),
                         dim3(static_cast<unsigned>(g)), dim3(kNarrowBlock), 0, s, rows, w, B, P,
                         acc_in, epi, W32, flags);
      return hipGetLastError();
    }
  }
  const int64_t grid = (P + kNarrowBlock * VW - 1) / (kNarrowBlock * VW);
  hipLaunchKernelGGL((k_reduce_narrow<U, VW, NT, NR, Epi>), dim3(static_cast<unsigned>(grid)),
                     dim3(kNarrowBlock), 0, s, rows, w, B, P, acc_in, epi, W32, flags);
  return hipGetLastError();
}

// Narrow k-unroll: selector 2 / 3 / 5 = 8 / 16 / 32, anything else = the
// per-P default.
int narrow_unroll(int flags, int64_t P) {
  switch ((flags & FEDAGG_UNROLL_MASK) >> FEDAGG_UNROLL_SHIFT) {
    case 2: return 8;
    case 3: return 16;
    case 5: return 32;
    default: return (P < kNarrowWideP || P >= kNarrowLongP) ? 8 : 16;
  }
}

template <int VW, bool NT, class NR, class Epi>
hipError_t launch_narrow_u(const NR& rows, const float* w, int64_t B, int64_t P,
                           const float* acc_in, const Epi& epi, float W32, int flags,
                           hipStream_t s) {
  switch (narrow_unroll(flags, P)) {
    case 8: return launch_narrow_t<8, VW, NT>(rows, w, B, P, acc_in, epi, W32, flags, s);
    case 32: return launch_narrow_t<32, VW, NT>(rows, w, B, P, acc_in, epi, W32, flags, s);
    default: return launch_narrow_t<16, VW, NT>(rows, w, B, P, acc_in, epi, W32, flags, s);
  }
}

// Plain reduce (EpiStore): NT from the flags.
template <class NR>
hipError_t launch_narrow_store(const NR& rows, int vw, const float* w, int64_t B, int64_t P,
                               const float* acc_in, float* out, float W32, int flags,
                               hipStream_t s) {
  const EpiStore st{out};
  const bool nt = (flags & FEDAGG_NT) != 0;
  if (vw == 4)
    return nt ? launch_narrow_u<4, true>(rows, w, B, P, acc_in, st, W32, flags, s)
              : launch_narrow_u<4, false>(rows, w, B, P, acc_in, st, W32, flags, s);
  if (vw == 2)
    return nt ? launch_narrow_u<2, true>(rows, w, B, P, acc_in, st, W32, flags, s)
              : launch_narrow_u<2, false>(rows, w, B, P, acc_in, st, W32, flags, s);
  return nt ? launch_narrow_u<1, true>(rows, w, B, P, acc_in, st, W32, flags, s)
            : launch_narrow_u<1, false>(rows, w, B, P, acc_in, st, W32, flags, s);
}

// Fused server step: non-temporal row loads.
template <class NR, class Epi>
hipError_t launch_narrow_step(const NR& rows, int vw, const float* w, int64_t B, int64_t P,
                              const float* acc_in, const Epi& epi, float W32, int flags,
                              hipStream_t s) {
  if (vw == 4) return launch_narrow_u<4, true>(rows, w, B, P, acc_in, epi, W32, flags, s);
  return vw == 2 ? launch_narrow_u<2, true>(rows, w, B, P, acc_in, epi, W32, flags, s)
                 : launch_narrow_u<1, true>(rows, w, B, P, acc_in, epi, W32, flags, s);
}


// FEDAGG_FAST: waves per workgroup for the split-K kernel (enough for ~4096
// waves), or 0 when one column per lane already gives a wave per SIMD: from
// there on the exact kernels are as fast or faster (tools/bench_fast.py:
// P = 199,210, K = 1000: exact 6.1 TB/s, split-K 5.1) and FEDAGG_FAST changes
// nothing.
int fast_split(int flags, int64_t P) {
  if (!(flags & FEDAGG_FAST)) return 0;
  const int64_t tiles = (P + 63) / 64;
  if (tiles >= 1024) return 0;
  int S = 2;
  while (S < 16 && tiles * S < 4096) S *= 2;
  return S;
}

template <class NR, class Epi>
hipError_t launch_splitk(const NR& rows, int S, const float* w, int64_t B, int64_t P,
                         const float* acc_in, const Epi& epi, float W32, int flags,
                         hipStream_t s) {
  const dim3 g(static_cast<unsigned>((P + 63) / 64));
  switch (S) {
    case 2:
      hipLaunchKernelGGL((k_reduce_splitk<2, 8, true, NR, Epi>), g, dim3(128), 0, s, rows, w, B,
                         P, acc_in, epi, W32, flags);
      break;
    case 4:
      hipLaunchKernelGGL((k_reduce_splitk<4, 8, true, NR, Epi>), g, dim3(256), 0, s, rows, w, B,
                         P, acc_in, epi, W32, flags);
      break;
    case 8:
      hipLaunchKernelGGL((k_reduce_splitk<8, 8, true, NR, Epi>), g, dim3(512), 0, s, rows, w, B,
                         P, acc_in, epi, W32, flags);
      break;
    default:
      hipLaunchKernelGGL((k_reduce_splitk<16, 8, true, NR, Epi>), g, dim3(1024), 0, s, rows, w,
                         B, P, acc_in, epi, W32, flags);
      break;
  }
  return hipGetLastError();
}

// Column-block widths the blocked kernels are built for (one workgroup's span
// of the wide mapping; a multiple of a narrow workgroup's kNarrowBlock * 4 columns).
inline bool valid_block_cols(int64_t C) { return C == 1024 || C == 2048 || C == 4096; }

// Validate a server step's operands and pack them for EpiStep.
int make_step(int algo, float coef, float* cloud, float* aux, float* avg_prev, float* buf,
              int momentum_init, float* grad, float* avg_out, const fedagg_sgd_params* sgd,
              StepPtrs* sp, bool* mom) {
  if (!sgd || !cloud) return FEDAGG_EINVAL;
  if (algo != FEDAGG_ALGO_FEDAVG && algo != FEDAGG_ALGO_ADABEST && algo != FEDAGG_ALGO_FEDDYN)
    return FEDAGG_EINVAL;
  if (algo != FEDAGG_ALGO_FEDAVG && !aux) return FEDAGG_EINVAL;
  *mom = sgd->momentum != 0.f;
  if (*mom && !buf) return FEDAGG_EINVAL;
  if (sgd->nesterov && (!*mom || sgd->one_minus_dampening != 1.f)) return FEDAGG_EINVAL;
  *sp = StepPtrs{cloud, aux, avg_prev, buf, grad, avg_out, coef,
                 SgdArgs{sgd->neg_lr, sgd->momentum, sgd->one_minus_dampening, sgd->weight_decay,
                         sgd->nesterov, sgd->maximize, momentum_init}};
  return 0;
}

bool step_aligned(const StepPtrs& p) {
  for (const float* q : {p.cloud, p.aux, p.avg_prev, p.buf, p.grad, p.avg_out})
    if (q && !aligned16(q)) return false;
  return true;
}

// f(EpiStep<ALGO, MOM>{sp}) for the runtime (algo, mom).
template <class F>
hipError_t with_step(int algo, bool mom, const StepPtrs& sp, F&& f) {
  switch (algo) {
    case FEDAGG_ALGO_FEDAVG:
      return mom ? f(EpiStep<FEDAGG_ALGO_FEDAVG, true>{sp})
                 : f(EpiStep<FEDAGG_ALGO_FEDAVG, false>{sp});
    case FEDAGG_ALGO_ADABEST:
      return mom ? f(EpiStep<FEDAGG_ALGO_ADABEST, true>{sp})
                 : f(EpiStep<FEDAGG_ALGO_ADABEST, false>{sp});
    case FEDAGG_ALGO_FEDDYN:
      return mom ? f(EpiStep<FEDAGG_ALGO_FEDDYN, true>{sp})
                 : f(EpiStep<FEDAGG_ALGO_FEDDYN, false>{sp});
    default:
      return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// FedDF teacher ensemble (fedsim/distributed/centralized/training/feddf.py
// :117-122): one nn.Linear layer of K stacked teacher models on the matrix
// cores.  y[k, m, n] = act(sum_i x[k, m, i] * W_k[n, i] + b_k[n]) with W_k /
// b_k read from teacher k's flat parameter vector (a row of the [K, P] slab,
// parameters_to_vector layout: W row-major [out, in], then b).
//
// A workgroup (4 waves) owns a 64-row x 64-column output tile of one
// teacher; x and W tiles of 32 inputs are staged through LDS (coalesced rows,
// zero-filled past the edges) and each wave runs 16 x 64 of the tile as four
// 16x16 accumulators of v_mfma_f32_16x16x4_f32 (exact f32: a k-ordered fmaf
// chain per output, the bias added last).  Every teacher's weights are read
// once per 64-row tile: a FedDF batch (64 samples) reads each teacher once.
// ---------------------------------------------------------------------------
constexpr int kTL_M = 64;  // output rows (samples) per workgroup
constexpr int kTL_N = 64;  // output columns (features) per workgroup
constexpr int kTL_K = 32;  // inputs per LDS stage
constexpr int kTL_PAD = 1;

constexpr int64_t kTL_WideIn = 1024;  // inputs above which a Linear layer counts as wide
constexpr size_t kTL_WidePadKB = 9;    // LDS reserved per workgroup of a wide layer: 6 per CU

// XCD-aware order of a 1-D grid of teacher tiles (the 1-D form of
// conv_tile_order below): launch index L runs on XCD L % 8, so in plain order
// the n_tiles x m_tiles tiles of one teacher land on up to eight XCDs and each
// fetches the teacher's input rows into its own L2 (SimpleCNN's fc: 8 output
// tiles, a 0.8 MB input per teacher).  Renumbered, each XCD walks one
// contiguous range of tiles, so a teacher's tiles share one L2.  Bijective;
// placement only changes speed, never results.
__device__ __forceinline__ uint32_t xcd_tile_1d() {
  const uint32_t L = blockIdx.x;
  const uint32_t n = gridDim.x, xcd = L & 7u, slot = L >> 3, q = n >> 3, r = n & 7u;
  return slot + (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q);
}

__global__ __launch_bounds__(256) void k_teacher_linear(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, int64_t M, int64_t in, int64_t out,
    float* __restrict__ y, int64_t n_tiles, int64_t m_tiles, int relu) {
  __shared__ float sx[kTL_M][kTL_K + kTL_PAD];
  __shared__ float sw[kTL_N][kTL_K + kTL_PAD];
  const int64_t tile = xcd_tile_1d();
  const int64_t k = tile / (n_tiles * m_tiles);
  const int64_t rem = tile - k * n_tiles * m_tiles;
  const int64_t m0 = (rem / n_tiles) * kTL_M;
  const int64_t n0 = (rem % n_tiles) * kTL_N;
  const float* xk = x + k * x_kstride;
  const float* wk = params + k * params_kstride + w_off;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // 64 x 32 of x and of W per stage: 2048 floats each, 8 per thread; 32
  // consecutive lanes read one row's 128 contiguous bytes.  The next stage's
  // loads are issued into registers before this stage's MFMAs, so their
  // latency hides behind the matrix work.
  float rx[8], rw[8];
  // 16-byte loads when every row of x and of this teacher's W starts 16-B
  // aligned (workgroup-uniform): thread t owns inputs 4 (t % 8) .. + 3 of
  // rows t / 8 + 32 j; else one float per load as e = t + 256 j
  const bool vec = (in % 4) == 0 && (reinterpret_cast<uintptr_t>(xk) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(wk) % 16) == 0;
  auto fetch = [&](int64_t i0) {
    if (vec) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = (t >> 3) + 32 * j;
        const int64_t i = i0 + 4 * (t & 7);
        const int64_t m = m0 + r;
        const int64_t n = n0 + r;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 vx = (m < M && i < in) ? *reinterpret_cast<const f32x4*>(xk + m * in + i) : z;
        const f32x4 vw = (n < out && i < in) ? *reinterpret_cast<const f32x4*>(wk + n * in + i) : z;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rx[4 * j + q] = vx[q];
          rw[4 * j + q] = vw[q];
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = t + 256 * j;
      const int r = e / kTL_K;
      const int64_t i = i0 + e % kTL_K;
      const int64_t m = m0 + r;
      const int64_t n = n0 + r;
      rx[j] = (m < M && i < in) ? xk[m * in + i] : 0.f;
      rw[j] = (n < out && i < in) ? wk[n * in + i] : 0.f;
    }
  };
  fetch(0);
  for (int64_t i0 = 0; i0 < in; i0 += kTL_K) {
    if (vec) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sx[(t >> 3) + 32 * j][4 * (t & 7) + q] = rx[4 * j + q];
          sw[(t >> 3) + 32 * j][4 * (t & 7) + q] = rw[4 * j + q];
        }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = t + 256 * j;
        sx[e / kTL_K][e % kTL_K] = rx[j];
        sw[e / kTL_K][e % kTL_K] = rw[j];
      }
    }
    __syncthreads();
    if (i0 + kTL_K < in) fetch(i0 + kTL_K);
    const int row = lane & 15;
    const int kk = lane >> 4;
#pragma unroll
    for (int s = 0; s < kTL_K / 4; ++s) {
      // A[row][k] = x[m0 + 16 wave + row][i0 + 4 s + k];  B[k][col] = W[n0 + 16 j + col][...]
      const float a = sx[wave * 16 + row][4 * s + kk];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float b = sw[j * 16 + row][4 * s + kk];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // C/D: col = lane & 15, row = (lane >> 4) * 4 + reg
  const float* bk = b_off >= 0 ? params + k * params_kstride + b_off : nullptr;
  float* yk = y + k * M * out;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + j * 16 + (lane & 15);
    if (n >= out) continue;
    const float bias = bk ? bk[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = m0 + wave * 16 + (lane >> 4) * 4 + r;
      if (m >= M) continue;
      float v = acc[j][r] + bias;
      if (relu) v = v < 0.f ? 0.f : v;  // torch.relu: keeps NaN and -0
      yk[m * out + n] = v;
    }
  }
}

// The same Linear tile with every staging load through a buffer descriptor
// (32-bit lane offsets fixed for the whole K loop, the stage advanced by the
// scalar offset, rows past M / out and the tail past ``in`` reading 0 from
// outside the descriptor's range).  The generic kernel above computes 64-bit
// addresses per load (101 VGPRs, 4 waves per SIMD): its 32-input stages then
// wait on memory with only one stage in flight (SimpleMLP's fc1: 212 us per
// 1000 teachers, 47 TFLOP/s).  Here the tile needs about half the registers,
// so twice the workgroups are resident to hide the same latency.  Same LDS
// layout and MFMA sequence: the same bits.  Taken when every teacher's x and
// W rows are 16-B aligned and the per-teacher extents fit 32-bit offsets.
__global__ __launch_bounds__(256) void k_teacher_linear_buf(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, int M, int in, int out,
    float* __restrict__ y, int n_tiles, int m_tiles, int relu) {
  __shared__ float sx[kTL_M][kTL_K + kTL_PAD];
  __shared__ float sw[kTL_N][kTL_K + kTL_PAD];
  const int tiles = n_tiles * m_tiles;
  const int tile = __builtin_amdgcn_readfirstlane(static_cast<int>(xcd_tile_1d()));
  const int k = tile / tiles;
  const int rem = tile - k * tiles;
  const int m0 = (rem / n_tiles) * kTL_M;
  const int n0 = (rem % n_tiles) * kTL_N;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  constexpr uint32_t kOut = 0x80000000u;  // > num_records: reads 0
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + int64_t(k) * x_kstride), static_cast<short>(0), M * in * 4,
      0x00020000);
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(params + int64_t(k) * params_kstride + w_off), static_cast<short>(0),
      out * in * 4, 0x00020000);
  // thread t stages inputs 4 (t % 8) .. + 3 of rows t / 8 and t / 8 + 32
  const int c4 = 4 * (t & 7);
  uint32_t xo[2], wo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (t >> 3) + 32 * j;
    xo[j] = (m0 + r < M) ? static_cast<uint32_t>(((m0 + r) * in + c4) * 4) : kOut;
    wo[j] = (n0 + r < out) ? static_cast<uint32_t>(((n0 + r) * in + c4) * 4) : kOut;
  }
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 rx[2], rw[2];
  auto fetch = [&](int i0) {
    const bool in_row = i0 + c4 < in;  // in % 4 == 0: the whole quad is in or out
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      rx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            xres, static_cast<int>(in_row ? xo[j] : kOut),
                                            i0 * 4, 0));
      rw[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            wres, static_cast<int>(in_row ? wo[j] : kOut),
                                            i0 * 4, 0));
    }
  };
  fetch(0);
  const int row = lane & 15;
  const int kk = lane >> 4;
  for (int i0 = 0; i0 < in; i0 += kTL_K) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sx[(t >> 3) + 32 * j][c4 + q] = rx[j][q];
        sw[(t >> 3) + 32 * j][c4 + q] = rw[j][q];
      }
    __syncthreads();
    if (i0 + kTL_K < in) fetch(i0 + kTL_K);
#pragma unroll
    for (int s4 = 0; s4 < kTL_K / 4; ++s4) {
      const float a = sx[wave * 16 + row][4 * s4 + kk];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float b = sw[j * 16 + row][4 * s4 + kk];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  const float* bk = b_off >= 0 ? params + int64_t(k) * params_kstride + b_off : nullptr;
  float* yk = y + int64_t(k) * M * out;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j * 16 + (lane & 15);
    if (n >= out) continue;
    const float bias = bk ? bk[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wave * 16 + (lane >> 4) * 4 + r;
      if (m >= M) continue;
      float v = acc[j][r] + bias;
      if (relu) v = v < 0.f ? 0.f : v;  // torch.relu: keeps NaN and -0
      yk[int64_t(m) * out + n] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// FedDF teacher ensemble, convolutional layers: one nn.Conv2d (groups 1,
// dilation 1, zero padding) of K stacked teachers as an implicit GEMM on the
// matrix cores.  Per teacher k the GEMM is
//     Y[oc][p] = sum_r W_k[oc][r] * X_k[r][p]      r = (c, kh, kw), p = (m, oh, ow)
// W_k is the conv weight exactly as it lies in the teacher's flat vector
// ([OC, C, KH, KW] row-major = [OC][R]); X_k is the im2col of the input,
// never materialised: each stage gathers RK reductions x 256 pixels of it
// from the input (L1/L2-resident: a 5x5 window reads each input element 25
// times) straight into LDS.  A workgroup (4 waves) owns 64 output channels x
// 256 pixels; a wave owns 64 x 64 as 2 x 2 tiles of v_mfma_f32_32x32x2_f32
// (one A and one B VGPR per 4096 flop, so LDS traffic stays far below the
// matrix rate).  The next stage's global loads are issued into registers
// before this stage's MFMAs.  Exact f32: each output is the r-ordered fmaf
// chain (zero-filled tail to a multiple of RK), then the bias, then ReLU.
// ---------------------------------------------------------------------------
// XCD-aware tile order for the teacher convolutions.  The hardware deals
// consecutive workgroups of a launch round-robin over the 8 XCDs (blocks b
// and b + 8 share one; MI355X_MICROARCH.md, workgroup dispatch), so in the
// plain (pixel tile, channel tile, teacher) order every teacher's tiles are
// spread over all 8 XCDs and its weights, and the images two neighbouring
// pixel tiles share, are fetched into up to eight L2s.  Renumbered, each
// XCD walks one contiguous range of the tile order: a teacher's weights are
// read from HBM about once, and the partial cache lines two neighbouring
// tiles write at an image boundary merge in one L2.  Bijective for any grid;
// placement only changes speed, never results.
struct ConvTile {
  int x, y, z;
};
__device__ __forceinline__ ConvTile conv_tile_order() {
  const uint32_t gx = gridDim.x, gy = gridDim.y;
  const uint32_t gxy = gx * gy, n = gxy * gridDim.z;
  const uint32_t L = blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z;
  const uint32_t xcd = L & 7u, slot = L >> 3, q = n >> 3, r = n & 7u;
  const uint32_t lg = slot + (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q);
  const uint32_t z = lg / gxy, rem = lg - z * gxy;
  const uint32_t y = rem / gx;
  // wave-uniform by construction; readfirstlane keeps the tile coordinates
  // (and the buffer descriptors built from them) in SGPRs
  return {__builtin_amdgcn_readfirstlane(int(rem - y * gx)), __builtin_amdgcn_readfirstlane(int(y)),
          __builtin_amdgcn_readfirstlane(int(z))};
}

constexpr int kTC_OC = 64;    // output channels per workgroup
constexpr int kTC_PX = 256;   // output pixels per workgroup (64 per wave)
constexpr int kTC_WPAD = 1;   // sW row pad: 32 lanes reading 32 rows hit 32 banks
constexpr int kTC_XPAD = 32;  // sX row pad: rows r and r+1 land on different bank halves

template <int RK>
__global__ __launch_bounds__(256) void k_teacher_conv2d(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, fedagg_conv2d_shape s,
    float* __restrict__ y, int relu) {
  __shared__ float sW[kTC_OC][RK + kTC_WPAD];
  __shared__ float sX[RK][kTC_PX + kTC_XPAD];
  // grid (pixel tiles, channel tiles, teachers): the tile coordinates come
  // from SGPRs, so the buffer resources below are wave-uniform (a descriptor
  // derived from a VALU division makes the compiler wrap every load in a
  // waterfall loop)
  const ConvTile tile = conv_tile_order();
  const int64_t k = tile.z;
  const int64_t oc0 = int64_t(tile.y) * kTC_OC;
  const int64_t px0 = int64_t(tile.x) * kTC_PX;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int64_t OHW = s.OH * s.OW;
  const int64_t NPX = s.M * OHW;
  const int64_t HW = s.H * s.W;
  const int64_t R = s.C * s.KH * s.KW;
  // the teacher's input and weight matrix as buffer resources: an offset past
  // num_records (the zero padding, the tails past R / OC / the last pixel)
  // reads 0 without a branch; per element the address is a 32-bit VGPR
  // offset, the (c, kh, kw) part of it wave-uniform
  constexpr uint32_t kOut = 0x80000000u;  // > num_records (host: < 2^31 bytes)
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + k * x_kstride), static_cast<short>(0),
      static_cast<int>(s.M * s.C * HW * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(params + k * params_kstride + w_off), static_cast<short>(0),
      static_cast<int>(s.OC * R * 4), 0x00020000);
  // this thread gathers pixel px0 + t of the tile
  const int64_t px = px0 + t;
  const bool px_ok = px < NPX;
  int ih0 = 0, iw0 = 0, vbase = 0;
  if (px_ok) {
    const int64_t m = px / OHW;
    const int64_t ohw = px - m * OHW;
    const int oh = static_cast<int>(ohw / s.OW);
    const int ow = static_cast<int>(ohw - int64_t(oh) * s.OW);
    ih0 = oh * static_cast<int>(s.stride_h) - static_cast<int>(s.pad_h);
    iw0 = ow * static_cast<int>(s.stride_w) - static_cast<int>(s.pad_w);
    vbase = static_cast<int>(m * s.C * HW) + ih0 * static_cast<int>(s.W) + iw0;
  }
  const int H = static_cast<int>(s.H), W = static_cast<int>(s.W);
  const int KH = static_cast<int>(s.KH), KW = static_cast<int>(s.KW);
  const int iHW = static_cast<int>(HW), iR = static_cast<int>(R);
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  constexpr int WPT = kTC_OC * RK / 256;  // weight elements per thread per stage
  float rw[WPT], rx[RK];
  auto fetch = [&](int r0) {
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = t + 256 * j;
      const int oc = static_cast<int>(oc0) + e / RK;
      const int r = r0 + e % RK;
      const uint32_t off = (oc < s.OC && r < iR) ? static_cast<uint32_t>(oc * iR + r) * 4u : kOut;
      rw[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            wres, static_cast<int>(off), 0, 0));
    }
    // wave-uniform walk of r = (c, kh, kw) through the stage
    int c = r0 / (KH * KW);
    const int rr = r0 - c * KH * KW;
    int kh = rr / KW;
    int kw = rr - kh * KW;
#pragma unroll
    for (int i = 0; i < RK; ++i) {
      const bool ok = px_ok && (r0 + i < iR) &&
                      static_cast<unsigned>(ih0 + kh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(iw0 + kw) < static_cast<unsigned>(W);
      const uint32_t off = ok ? static_cast<uint32_t>(vbase + c * iHW + kh * W + kw) * 4u : kOut;
      rx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            xres, static_cast<int>(off), 0, 0));
      if (++kw == KW) {
        kw = 0;
        if (++kh == KH) {
          kh = 0;
          ++c;
        }
      }
    }
  };
  fetch(0);
  for (int r0 = 0; r0 < iR; r0 += RK) {
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = t + 256 * j;
      sW[e / RK][e % RK] = rw[j];
    }
#pragma unroll
    for (int i = 0; i < RK; ++i) sX[i][t] = rx[i];
    __syncthreads();
    if (r0 + RK < iR) fetch(r0 + RK);
    const int col = lane & 31;
    const int kk = lane >> 5;
#pragma unroll
    for (int st = 0; st < RK / 2; ++st) {
      // A[i][k] = W[oc0 + 32 a + i][r0 + 2 st + k];  B[k][j] = X[r0 + 2 st + k][64 wave + 32 b + j]
      const float a0 = sW[col][2 * st + kk];
      const float a1 = sW[32 + col][2 * st + kk];
      const float b0 = sX[2 * st + kk][wave * 64 + col];
      const float b1 = sX[2 * st + kk][wave * 64 + 32 + col];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D of 32x32: col = lane & 31 (pixel), row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5) (channel)
  const float* bk = b_off >= 0 ? params + k * params_kstride + b_off : nullptr;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int64_t p = px0 + wave * 64 + b * 32 + (lane & 31);
    if (p >= NPX) continue;
    const int64_t m = p / OHW;
    float* yp = y + (k * s.M + m) * s.OC * OHW + (p - m * OHW);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t oc = oc0 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (oc >= s.OC) continue;
        float v = acc[a][b][e] + (bk ? bk[oc] : 0.f);
        if (relu) v = v < 0.f ? 0.f : v;  // torch.relu: keeps NaN and -0
        yp[oc * OHW] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The same convolution with the input tile resident in LDS (stride 1, square
// KS x KS kernels: every Conv2d of the reference's CNNs, 5 x 5).  The gather
// above spends ~20 address instructions per im2col element, more issue slots
// than its MFMAs get; here a workgroup stages, per chunk of CC input
// channels, the zero-padded planes of the (at most nslot) images its 256
// output pixels fall in, [nslot][CC][Hp][Wp], plus the chunk's weights in
// their own layout, [64 oc][CC * KS * KS] (odd row pitch: 32 rows hit 32
// banks).  An MFMA operand is then ONE ds_read_b32 at a per-lane base + an
// immediate offset: the k pair of v_mfma_f32_32x32x2_f32 is two adjacent
// channels (kk = lane >> 5 is folded into the per-lane base), the tap (kh, kw)
// and the channel pair are the immediate.  Chain order per output (restated
// by oracle/fedagg_ref.c ref_teacher_conv2d_f32 with cc = CC): channel
// chunks, then kh, then channel pairs, then kw, then the pair's two channels;
// channels past C (C odd) are zero terms.  The chunk's planes and weights
// are loaded into registers while the previous chunk's MFMAs run; the halo
// of the planes is zeroed once and never written.  Offsets for the plane
// staging are decoded once per thread (packed: global << 0 | LDS << 18).
// ---------------------------------------------------------------------------
constexpr int kTC_XPK_LDS = 14;  // LDS float index bits of a packed staging offset
constexpr int kTC_XPK_GLB = 18;  // global float offset bits

template <int KS, int CC, int XM>
__device__ __forceinline__ void conv2d_lds_tile(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, const fedagg_conv2d_shape& s, int nslot,
    float* __restrict__ y, int relu) {
  constexpr int TAPS = KS * KS;
  constexpr int RC = TAPS * CC;  // reductions per chunk
  constexpr int RW = RC + 1;     // sW row pitch (odd)
  constexpr int WPT = (RC + 3) / 4;  // weight columns per thread per chunk
  extern __shared__ float lds[];
  float* sW = lds;
  float* sX = lds + kTC_OC * RW;
  // grid (pixel tiles, channel tiles, teachers): tile coordinates straight
  // from the SGPRs, so the buffer descriptors below are provably uniform (one
  // derived from a VALU division costs a waterfall loop per load)
  const ConvTile tile = conv_tile_order();
  const int64_t k = tile.z;
  const int oc0 = tile.y * kTC_OC;
  const int pxt = tile.x;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int C = static_cast<int>(s.C), H = static_cast<int>(s.H), W = static_cast<int>(s.W);
  const int OW = static_cast<int>(s.OW);
  const int OHW = static_cast<int>(s.OH * s.OW);
  const int Hp = static_cast<int>(s.OH) + KS - 1, Wp = OW + KS - 1, HpWp = Hp * Wp;
  const int HW = H * W;
  const int NPX = static_cast<int>(s.M) * OHW;
  const int R = C * TAPS;
  const int OC = static_cast<int>(s.OC);
  const int px0 = pxt * kTC_PX;
  const int m_lo = px0 / OHW;  // first image of the tile (VGPR: offsets only)
  const int pt = static_cast<int>(s.pad_h), pl = static_cast<int>(s.pad_w);
  // the images of this tile (reads past the teacher's last image are 0) and
  // the teacher's [OC][C][KS][KS] weights
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + k * x_kstride), static_cast<short>(0),
      static_cast<int>(s.M * C * HW * 4), 0x00020000);
  const uint32_t x_tile4 = static_cast<uint32_t>(m_lo * C * HW) * 4u;
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(params + k * params_kstride + w_off), static_cast<short>(0),
      OC * R * 4, 0x00020000);
  const int plane_n = nslot * HW;  // staged elements per channel of a chunk
  const int xtot = CC * plane_n;
  // plane staging: element e = t + 256 i of a chunk is (channel cl, slot,
  // hw), cl slowest; packed: its global float offset from the tile's first
  // image (channel c0 added per chunk as the scalar offset) and its LDS index
  uint32_t xpk[XM];
#pragma unroll
  for (int i = 0; i < XM; ++i) {
    const int e = t + 256 * i;
    if (e < xtot) {
      const int cl = e / plane_n;
      const int rem = e - cl * plane_n;
      const int slot = rem / HW;
      const int hw = rem - slot * HW;
      const int h = hw / W;
      const int w = hw - h * W;
      const uint32_t g = static_cast<uint32_t>(slot * C * HW + cl * HW + hw);
      const uint32_t l = static_cast<uint32_t>(((slot * CC + cl) * Hp + h + pt) * Wp + w + pl);
      xpk[i] = g | (l << kTC_XPK_GLB);
    } else {
      xpk[i] = 0xffffffffu;
    }
  }
  for (int i = t; i < nslot * CC * HpWp; i += 256) sX[i] = 0.f;
  __syncthreads();  // the halo zeroes land before any thread stages a plane
  // weight staging: thread t owns output channel oc0 + t / 4 and the chunk
  // columns j = t % 4 + 4 i (one VGPR base, immediate offsets); rows past OC
  // read 0 through the descriptor's range
  const int wq = t & 3;
  const uint32_t wg4 = static_cast<uint32_t>((oc0 + (t >> 2)) * R + wq) * 4u;
  const int wl = (t >> 2) * RW + wq;
  float rw[WPT], rx[XM];
  auto fetch = [&](int c0) {
    const int soff_w = c0 * TAPS * 4;
    const int soff_x = c0 * HW * 4;
    if (C - c0 >= CC) {  // a full chunk (every chunk unless C is odd)
#pragma unroll
      for (int i = 0; i < WPT; ++i)
        rw[i] = (wq + 4 * i < RC)
                    ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    wres, static_cast<int>(wg4 + 16u * i), soff_w, 0))
                    : 0.f;
#pragma unroll
      for (int i = 0; i < XM; ++i) {
        const uint32_t g4 = (xpk[i] & ((1u << kTC_XPK_GLB) - 1u)) * 4u + x_tile4;
        rx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              xres, static_cast<int>(g4), soff_x, 0));
      }
    } else {  // the last chunk of an odd C: channels past C are zero terms
      const int jlim = (C - c0) * TAPS;
      const int xlim = (C - c0) * plane_n;
#pragma unroll
      for (int i = 0; i < WPT; ++i)
        rw[i] = (wq + 4 * i < RC && wq + 4 * i < jlim)
                    ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    wres, static_cast<int>(wg4 + 16u * i), soff_w, 0))
                    : 0.f;
#pragma unroll
      for (int i = 0; i < XM; ++i) {
        const uint32_t g4 = (xpk[i] & ((1u << kTC_XPK_GLB) - 1u)) * 4u + x_tile4;
        rx[i] = (t + 256 * i < xlim)
                    ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    xres, static_cast<int>(g4), soff_x, 0))
                    : 0.f;
      }
    }
  };
  // operand bases: A = weights (oc = lane & 31 [+ 32], channel + kk), B =
  // the staged planes at this lane's output pixel (channel + kk)
  const int col = lane & 31;
  const int kk = lane >> 5;
  const int wa = col * RW + kk * TAPS;
  int xb[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    int p = px0 + wave * 64 + b * 32 + col;
    p = p < NPX ? p : NPX - 1;
    const int m = p / OHW;
    const int ohw = p - m * OHW;
    const int oh = ohw / OW;
    const int ow = ohw - oh * OW;
    xb[b] = ((m - m_lo) * CC + kk) * HpWp + oh * Wp + ow;
  }
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  fetch(0);
  for (int c0 = 0; c0 < C; c0 += CC) {
#pragma unroll
    for (int i = 0; i < WPT; ++i)
      if (wq + 4 * i < RC) sW[wl + 4 * i] = rw[i];
#pragma unroll
    for (int i = 0; i < XM; ++i)
      if (xpk[i] != 0xffffffffu) sX[xpk[i] >> kTC_XPK_GLB] = rx[i];
    __syncthreads();
    if (c0 + CC < C) fetch(c0 + CC);
#pragma unroll
    for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
      for (int cp = 0; cp < CC / 2; ++cp) {
        const float* pb0 = sX + xb[0] + 2 * cp * HpWp + kh * Wp;
        const float* pb1 = sX + xb[1] + 2 * cp * HpWp + kh * Wp;
        const float* pa = sW + wa + 2 * cp * TAPS + kh * KS;
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const float a0 = pa[kw];
          const float a1 = pa[32 * RW + kw];
          const float b0 = pb0[kw];
          const float b1 = pb1[kw];
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  const float* bk = b_off >= 0 ? params + k * params_kstride + b_off : nullptr;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int p = px0 + wave * 64 + b * 32 + col;
    if (p >= NPX) continue;
    const int m = p / OHW;
    float* yp = y + (k * s.M + m) * s.OC * OHW + (p - m * OHW);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int oc = oc0 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * kk;
        if (oc >= OC) continue;
        float v = acc[a][b][e] + (bk ? bk[oc] : 0.f);
        if (relu) v = v < 0.f ? 0.f : v;  // torch.relu: keeps NaN and -0
        yp[int64_t(oc) * OHW] = v;
      }
    }
  }
}

// Compiled for 3 waves per SIMD (4 spill 57 VGPRs: SimpleCNN2 conv2 7.50 vs
// 6.92 ms, profiles/r02xi) ...
template <int KS, int CC, int XM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_teacher_conv2d_lds(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, fedagg_conv2d_shape s, int nslot,
    float* __restrict__ y, int relu) {
  conv2d_lds_tile<KS, CC, XM>(x, x_kstride, params, params_kstride, w_off, b_off, s, nslot, y, relu);
}

// ... except chunks of 2 channels with 8 staging registers, which fit 4 waves
// per SIMD in 128 VGPRs (16 B of scratch): SimpleCNN's conv2 3.632 -> 3.535 ms
// per 500 teachers, same bits (profiles/r04s/; XM = 16 would spill 100 B)
template <int KS, int CC, int XM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_teacher_conv2d_lds4(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, fedagg_conv2d_shape s, int nslot,
    float* __restrict__ y, int relu) {
  conv2d_lds_tile<KS, CC, XM>(x, x_kstride, params, params_kstride, w_off, b_off, s, nslot, y, relu);
}

// ---------------------------------------------------------------------------
// The LDS-resident convolution for inputs of few channels (CI = 1 or 3: the
// first conv of the reference's CNNs, grayscale and RGB).  The chunked
// kernel above pairs two CHANNELS per MFMA k step, so CI = 3 runs as 4
// channels and CI = 1 as 2: a third / half of its matrix-core work is zero
// terms.  Here every channel is staged at once and the k pairs run over the
// flattened reduction index r = (c, kh, kw): ceil(CI*KS*KS / 2) steps, one
// zero term at most (a zero weight times a zero register: exact).  The k
// pair of a lane differs in its plane offset, chosen per step from two
// compile-time constants.  Chain order = the natural (c, kh, kw) order
// (fedagg_conv_order 0, oracle ref_teacher_conv2d_f32 with cc = 0): a
// trailing +0 term leaves a chain that never holds -0 unchanged.
// ---------------------------------------------------------------------------
// 4 waves per workgroup of the flat conv, 64 output pixels each (8 stage
// each image once per 512 pixels but run two workgroups per CU: conv1 2.33
// vs 2.13 ms, profiles/r02xf); compiled for 5 waves per SIMD (4 -> 3 lost 10 %,
// r02x3; with the compact row staging 5 fit without spills in <= 96 VGPRs:
// SimpleCNN2 conv1 2.058 vs 2.217 ms, profiles/r03l; 6 spill)
constexpr int kFlatThreads = 64 * 4;
// POOL: the 2 x 2 / stride 2 max pool (padding ppad = 0 or 1) that follows
// the layer is fused into the store (FEDAGG_CONV_MAXPOOL2; SimpleCNN's
// relu -> max_pool2d(2, 2, padding=1), simple_models.py:156-159).  The
// tile's pixel slots then run over (image, pooled row, pooled column, window
// member) with the member fastest, so the four conv outputs of one window
// sit in one quad of lanes (the MFMA result's pixel dimension is the lane):
// two DPP quad swaps combine them in window order with max_pool2d's rule
// (take v if v > m or v is NaN; members in the padding are -inf), and one
// lane per quad stores the pooled value.  The conv values are the unfused
// kernel's bits, so the result is the conv + pool pass bit for bit; only
// the pooled [OC, PH, PW] planes are written.
template <int CTRL>
__device__ __forceinline__ float pool_dpp_max(float m) {
  // m combined with the value of the quad partner selected by CTRL (a LATER
  // window member for the lanes whose result is used)
  const float v = __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, m), CTRL, 0xF, 0xF, false));
  return (v > m || __builtin_isnan(v)) ? v : m;
}

template <int KS, int CI, int XM, bool HALF, bool POOL>
__global__ __launch_bounds__(kFlatThreads) __attribute__((amdgpu_waves_per_eu(5, 5))) void k_teacher_conv2d_flat(
    const float* __restrict__ x, int64_t x_kstride, const float* __restrict__ params,
    int64_t params_kstride, int64_t w_off, int64_t b_off, fedagg_conv2d_shape s, int nslot,
    int nrows, float* __restrict__ y, int relu, int ppad) {
  constexpr int TAPS = KS * KS;
  constexpr int R = CI * TAPS;
  constexpr int RP = (R + 1) / 2;    // k steps
  constexpr int RW = 2 * RP + 1;     // sW row pitch (odd)
  constexpr int WPT = (2 * RP + 3) / 4;
  // HALF (OC <= 32: the upper 32 output channels of the MFMA tile do not
  // exist): the second accumulator pair takes two more 32-pixel groups
  // instead, so a wave owns 128 pixels and the tile 512
  constexpr int NPG = HALF ? 4 : 2;          // 32-pixel groups per wave
  constexpr int TPX = 32 * NPG * (kFlatThreads / 64);
  extern __shared__ float lds[];
  float* sW = lds;
  float* sX = lds + kTC_OC * RW;
  // plain dispatch order here: this kernel's input is shared by every
  // teacher and its weights are a few KB, so the XCD order (conv_tile_order)
  // has nothing to save, and it measured 2 % slower on SimpleCNN2's conv1
  // (2.249 vs 2.198 ms at K=500, the two builds interleaved, profiles/r03pmc/)
  const int64_t k = blockIdx.z;
  const int oc0 = blockIdx.y * kTC_OC;
  const int pxt = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int H = static_cast<int>(s.H), W = static_cast<int>(s.W);
  const int OW = static_cast<int>(s.OW);
  const int OHW = static_cast<int>(s.OH * s.OW);
  const int Hp = static_cast<int>(s.OH) + KS - 1, Wp = OW + KS - 1;
  const int HW = H * W;
  const int OH = static_cast<int>(s.OH);
  // pooled planes (POOL): PH x PW windows of 2 x 2, four pixel slots each
  const int PH = POOL ? (OH + 2 * ppad - 2) / 2 + 1 : 1;
  const int PW = POOL ? (OW + 2 * ppad - 2) / 2 + 1 : 1;
  const int PHW = PH * PW;
  // pixel slots of the launch: conv pixels, or (window, member) pairs
  const int NPX = static_cast<int>(s.M) * (POOL ? 4 * PHW : OHW);
  const int OC = static_cast<int>(s.OC);
  const int px0 = pxt * TPX;
  const int m_lo = POOL ? (px0 >> 2) / PHW : px0 / OHW;
  const int pt = static_cast<int>(s.pad_h), pl = static_cast<int>(s.pad_w);
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + k * x_kstride), static_cast<short>(0),
      static_cast<int>(s.M * CI * HW * 4), 0x00020000);
  const uint32_t x_tile4 = static_cast<uint32_t>(m_lo * CI * HW) * 4u;
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(params + k * params_kstride + w_off), static_cast<short>(0),
      OC * R * 4, 0x00020000);
  // stage every channel of the tile's images: element e = t + 256 i is
  // (slot, channel, hw) in the input's own order, i.e. global offset e.
  // Only the padded rows the tile's output rows read are staged (and
  // zeroed): from row_lo of the first image to row_hi of the last one
  // (a 256-pixel tile needs ~1/3 of the two 24 x 24 images it touches).
  // In LDS they are packed per channel as stacked padded rows g = slot * Hp
  // + row, from g = row_lo on: sX[c][g - row_lo][col], ``nrows`` rows per
  // channel (the host's bound for any tile), so the workgroup's LDS holds
  // only those rows and more workgroups fit on a CU.
  const int CP = nrows * Wp;  // channel pitch in sX
  const int pend = (px0 + TPX < NPX ? px0 + TPX : NPX) - 1;
  // slot of the tile's last image; the padded rows its pixels read (POOL:
  // whole images, a window's rows straddle the tile's first / last row)
  const int last = (POOL ? (pend >> 2) / PHW : pend / OHW) - m_lo;
  const int row_lo = POOL ? 0 : (px0 - m_lo * OHW) / OW;
  const int row_hi = POOL ? Hp - 1 : (pend - (m_lo + last) * OHW) / OW + KS - 1;
  const int nrow = last * Hp + row_hi - row_lo + 1;  // rows this tile stages (<= nrows)
  // after the staged rows: four dump slots per thread (sX[CI * CP + 4 t ..],
  // for elements the tile does not need), then the tile's biases
  float* sBias = sX + CI * CP + 4 * kFlatThreads;
  for (int c = 0; c < CI; ++c)
    for (int q = t; q < nrow * Wp; q += kFlatThreads) sX[c * CP + q] = 0.f;
  constexpr uint32_t kOut = 0x80000000u;  // past every descriptor: loads 0, stores dropped
  // (slot, channel, row, column) of each staged element (group), stepped by
  // the mixed-radix digits of the per-load step (wave-uniform) instead of
  // three divisions per element; one the tile does not need loads 0 and is
  // written to the thread's dump slots, so neither phase branches per lane.
  // A staged element sits in stacked padded row g = slot * Hp + h + pt; the
  // tile needs rows row_lo .. last * Hp + row_hi, i.e. g - row_lo < nrow
  // (an element of an image past the tile's last is past row_hi of the last slot).
  const int g0 = pt - row_lo;
  // V4 (rows a multiple of 4 wide, 16-B aligned input: the reference models'
  // 24- and 28-wide images): groups of 4 elements of one row per 16-byte
  // load, stepped by the digits of 4 x kFlatThreads; else single elements
  const bool v4 = (W & 3) == 0 && (x_kstride & 3) == 0 &&
                  (reinterpret_cast<uintptr_t>(x) & 15) == 0;  // wave-uniform
  const int NE = v4 ? 4 : 1;  // elements per load
  const int step = NE * kFlatThreads;
  const int dW = step % W, qW = step / W;
  const int dH = qW % H, qH = qW / H;
  const int dC = qH % CI, dS = qH / CI;
  const int e0 = NE * t;
  int ew = e0 % W, eh = (e0 / W) % H, ec = (e0 / W / H) % CI, es = e0 / W / H / CI;
  float rx[XM];
  int lidx[XM];
  auto locate = [&](int i) {  // LDS index (or the dump) and load offset of load i
    const int e = e0 + step * i;
    const int gr = __mul24(es, Hp) + eh + g0;  // staged row, from row_lo
    const bool need = static_cast<unsigned>(gr) < static_cast<unsigned>(nrow);
    lidx[i] = need ? __mul24(ec, CP) + __mul24(gr, Wp) + ew + pl : CI * CP + NE * t;
    const uint32_t off = need ? e * 4u + x_tile4 : kOut;
    ew += dW;
    int cy = ew >= W;
    ew -= cy ? W : 0;
    eh += dH + cy;
    cy = eh >= H;
    eh -= cy ? H : 0;
    ec += dC + cy;
    cy = ec >= CI;
    ec -= cy ? CI : 0;
    es += dS + cy;
    return static_cast<int>(off);
  };
  if (v4) {
#pragma unroll
    for (int i = 0; i < XM / 4; ++i) {
      const f32x4 v = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, locate(i), 0, 0));
#pragma unroll
      for (int q = 0; q < 4; ++q) rx[4 * i + q] = v[q];
    }
  } else {
#pragma unroll
    for (int i = 0; i < XM; ++i)
      rx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xres, locate(i), 0, 0));
  }
  // this tile's biases (0 past OC, or without a bias), read back per output channel
  if (t < kTC_OC) {
    const int oc = oc0 + t;
    sBias[t] = (b_off >= 0 && oc < OC) ? params[k * params_kstride + b_off + oc] : 0.f;
  }
  // weights: thread t owns output channel oc0 + t / 4, columns t % 4 + 4 i
  // (columns past R, and rows past OC, are zero)
  const int wq = t & 3;
  const uint32_t wg4 = static_cast<uint32_t>((oc0 + (t >> 2)) * R + wq) * 4u;
  const int wl = (t >> 2) * RW + wq;
  float rw[WPT];
#pragma unroll
  for (int i = 0; i < WPT; ++i)
    rw[i] = (t < 256 && wq + 4 * i < R) ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     wres, static_cast<int>(wg4 + 16u * i), 0, 0))
                             : 0.f;
  __syncthreads();  // halo zeroes before the planes land
  if (v4) {
#pragma unroll
    for (int i = 0; i < XM / 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) sX[lidx[i] + q] = rx[4 * i + q];
  } else {
#pragma unroll
    for (int i = 0; i < XM; ++i) sX[lidx[i]] = rx[i];
  }
#pragma unroll
  for (int i = 0; i < WPT; ++i)
    if (t < 256 && wq + 4 * i < 2 * RP) sW[wl + 4 * i] = rw[i];
  __syncthreads();
  const int col = lane & 31;
  const int kk = lane >> 5;
  const float* pa = sW + col * RW + kk;
  int xb[NPG];
#pragma unroll
  for (int b = 0; b < NPG; ++b) {
    int p = px0 + wave * 32 * NPG + b * 32 + col;
    p = p < NPX ? p : NPX - 1;
    int m, oh, ow;
    if constexpr (POOL) {  // window q, member d: conv pixel (2i - ppad + d/2, 2j - ppad + d%2)
      const int q = p >> 2, d = p & 3;
      m = q / PHW;
      const int ij = q - m * PHW;
      const int i = ij / PW;
      oh = 2 * i - ppad + (d >> 1);
      ow = 2 * (ij - i * PW) - ppad + (d & 1);
      oh = oh < 0 ? 0 : oh >= OH ? OH - 1 : oh;  // padding members: any pixel (masked)
      ow = ow < 0 ? 0 : ow >= OW ? OW - 1 : ow;
    } else {
      m = p / OHW;
      const int ohw = p - m * OHW;
      oh = ohw / OW;
      ow = ohw - oh * OW;
    }
    xb[b] = ((m - m_lo) * Hp + oh - row_lo) * Wp + ow;
  }
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
#pragma unroll
  for (int st = 0; st < RP; ++st) {
    const int r0 = 2 * st, r1 = 2 * st + 1;
    const int o0 = (r0 / TAPS) * CP + ((r0 % TAPS) / KS) * Wp + r0 % KS;
    const int o1 = r1 < R ? (r1 / TAPS) * CP + ((r1 % TAPS) / KS) * Wp + r1 % KS : 0;
    const int ob = kk ? o1 : o0;
    const float a0 = pa[2 * st];
    float bv[NPG];
#pragma unroll
    for (int b = 0; b < NPG; ++b) bv[b] = sX[xb[b] + ob];
    if (r1 >= R && kk) {  // the zero term of an odd R
#pragma unroll
      for (int b = 0; b < NPG; ++b) bv[b] = 0.f;
    }
    if constexpr (HALF) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[g >> 1][g & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv[g], acc[g >> 1][g & 1], 0, 0, 0);
    } else {
      const float a1 = pa[32 * RW + 2 * st];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv[0], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv[1], acc[0][1], 0, 0, 0);
      // the upper 32 output channels unconditionally: a tile with fewer
      // than 33 channels reads zero weights there and never stores them, and
      // a branch per k step kept the compiler from issuing the next step's
      // LDS reads under this step's MFMAs
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv[0], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv[1], acc[1][1], 0, 0, 0);
    }
  }
  // epilogue: buffer stores into this teacher's output, the lane's pixel in
  // the VGPR offset (kOut: a pixel past the launch, a channel past OC, a
  // non-leader lane of a pooled window -- the store is dropped), the output
  // channel's plane in the scalar offset; the bias from LDS.  No per-lane
  // branch, no 64-bit address per store.
  const int PLANE = POOL ? PHW : OHW;  // per output channel
  const __amdgpu_buffer_rsrc_t yres = __builtin_amdgcn_make_buffer_rsrc(
      y + k * s.M * s.OC * PLANE, static_cast<short>(0), static_cast<int>(s.M * s.OC * PLANE * 4),
      0x00020000);
  uint32_t yoff[NPG];
  bool inside[NPG];
#pragma unroll
  for (int b = 0; b < NPG; ++b) {
    const int p = px0 + wave * 32 * NPG + b * 32 + col;
    const bool pin = p < NPX;
    const int pc = pin ? p : 0;
    int m, pix;
    if constexpr (POOL) {
      // a quad of lanes holds one window's members in order; all four lanes
      // of a quad are in or out of the launch together (NPX is a multiple of 4)
      const int q = pc >> 2, d = pc & 3;
      m = q / PHW;
      pix = q - m * PHW;
      const int i = pix / PW;
      const int oh = 2 * i - ppad + (d >> 1);
      const int ow = 2 * (pix - i * PW) - ppad + (d & 1);
      inside[b] = oh >= 0 && oh < OH && ow >= 0 && ow < OW;
    } else {
      m = pc / OHW;
      pix = pc - m * OHW;
      inside[b] = true;
    }
    const bool store = pin && (!POOL || (col & 3) == 0);
    yoff[b] = store ? static_cast<uint32_t>((m * OC + 4 * kk) * PLANE + pix) * 4u : kOut;
  }
  // FULL: every channel of the tile exists (the common case, no channel test)
  auto epilogue = [&](auto full) {
    constexpr bool FULL = decltype(full)::value;
#pragma unroll
    for (int a = 0; a < (HALF ? 1 : 2); ++a) {
      float bias[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if ((e & 3) == 0) {  // read four at a time: one LDS wait per 4 channels
#pragma unroll
          for (int j = 0; j < 4; ++j) bias[e + j] = sBias[a * 32 + j + 2 * e + 4 * kk];
        }
        const int ocr = a * 32 + (e & 3) + 8 * (e >> 2);  // + 4 kk: this lane's channel
        if (!FULL && oc0 + ocr >= OC) continue;  // wave-uniform: both halves past OC
        const bool cok = FULL || oc0 + ocr + 4 * kk < OC;
        const uint32_t soff = static_cast<uint32_t>((oc0 + ocr) * PLANE) * 4u;
#pragma unroll
        for (int b = 0; b < NPG; ++b) {
          float v = (HALF ? acc[b >> 1][b & 1][e] : acc[a][b & 1][e]) + bias[e];
          if (relu) v = v < 0.f ? 0.f : v;  // torch.relu: keeps NaN and -0
          if constexpr (POOL) {
            if (!inside[b]) v = -__builtin_huge_valf();
            v = pool_dpp_max<0xB1>(v);  // members (0, 1) and (2, 3): quad_perm [1, 0, 3, 2]
            v = pool_dpp_max<0x4E>(v);  // then (01, 23): quad_perm [2, 3, 0, 1]
          }
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), yres,
                                                static_cast<int>(cok ? yoff[b] : kOut),
                                                static_cast<int>(soff), 0);
        }
      }
    }
  };
  if (oc0 + (HALF ? 32 : kTC_OC) <= OC)
    epilogue(std::true_type{});
  else
    epilogue(std::false_type{});
}

// Launch plan of k_teacher_conv2d_lds for a shape, or false (the gather
// kernel runs it).  cc: channels per chunk, xm: staging registers per
// thread, nslot: images a 256-pixel tile can touch, lds: bytes.
struct ConvLdsPlan {
  int ks, cc, xm, nslot;
  int nrows;  // flat kernel: stacked padded rows staged per channel
  size_t lds;
};

bool conv_lds_plan(const fedagg_conv2d_shape& s, ConvLdsPlan* p, int pool_pad = -1) {
  if (s.KH != s.KW || (s.KH != 5 && s.KH != 3) || s.stride_h != 1 || s.stride_w != 1) return false;
  const int64_t ks = s.KH;
  const int64_t Hp = s.OH + ks - 1, Wp = s.OW + ks - 1;
  if (s.H + s.pad_h > Hp || s.W + s.pad_w > Wp) return false;  // input rows past the window
  const int64_t OHW = s.OH * s.OW, HW = s.H * s.W;
  if (s.M * OHW >= (int64_t(1) << 31)) return false;
  int64_t nslot = (kTC_PX - 2) / OHW + 2;
  if (nslot > s.M) nslot = s.M;
  if (s.C == 1 || s.C == 3) {  // every channel staged at once (k_teacher_conv2d_flat)
    const int64_t tpx = (s.OC <= 32 ? 2 : 1) * kFlatThreads;  // HALF tiles: 512 pixels
    // images a tile touches: tpx pixels, or tpx / 4 pooled windows (POOL)
    const int64_t per_img = pool_pad >= 0 ? ((s.OH + 2 * pool_pad - 2) / 2 + 1) *
                                                ((s.OW + 2 * pool_pad - 2) / 2 + 1)
                                          : OHW;
    const int64_t per_tile = pool_pad >= 0 ? tpx / 4 : tpx;
    int64_t fslot = (per_tile - 2) / per_img + 2;
    if (fslot > s.M) fslot = s.M;
    const int64_t xall = s.C * fslot * HW;
    // one teacher's output is stored through a buffer descriptor (31-bit offsets)
    const bool y_fits = s.M * s.OC * per_img * 4 < (int64_t(1) << 31);
    if (xall <= 16 * kFlatThreads && y_fits) {
      const int64_t rw = (s.C * ks * ks + 1) / 2 * 2 + 1;
      // rows a tile reads: its output rows (a run of tpx pixels meets at most
      // ceil((tpx - 1) / OW) + 1 of them; image boundaries are row
      // boundaries) plus KS - 1 halo rows per image; POOL stages whole images
      int64_t nrows = fslot * Hp;
      if (pool_pad < 0) {
        const int64_t rows_out = (tpx - 1 + s.OW - 1) / s.OW + 1;
        if (rows_out + fslot * (ks - 1) < nrows) nrows = rows_out + fslot * (ks - 1);
      }
      p->ks = static_cast<int>(ks);
      p->cc = 0;
      p->xm = xall <= 8 * kFlatThreads ? 8 : 16;
      p->nslot = static_cast<int>(fslot);
      p->nrows = static_cast<int>(nrows);
      // weights, the staged rows, four dump slots per thread, the tile's biases
      p->lds = static_cast<size_t>(kTC_OC * rw + s.C * nrows * Wp + 4 * kFlatThreads + kTC_OC) *
               sizeof(float);
      if (p->lds <= 64 * 1024) return true;
    }
  }
  if (pool_pad >= 0) return false;  // the pool is fused by the flat kernel only
  // chunks of 2 channels: with 8 staging registers the kernel runs at 4
  // waves per SIMD (k_teacher_conv2d_lds4), which beats chunks of 4 at 3
  // (SimpleCNN2 conv2 6.973 -> 6.856 ms, SimpleCNN conv2 3.632 -> 3.535 ms
  // per 500 teachers, profiles/r04s, r04u; at 3 waves chunks of 4 had led
  // where they fit 8 registers, and 2 where 4 needed 16: profiles/r02xa)
  const int cc = 2;
  const int64_t xtot = cc * nslot * HW;
  const int xm = xtot <= 8 * 256 ? 8 : 16;
  if (xtot > xm * 256) return false;
  if (nslot * cc * Hp * Wp >= (int64_t(1) << kTC_XPK_LDS)) return false;
  if (nslot * s.C * HW + cc * HW >= (int64_t(1) << kTC_XPK_GLB)) return false;
  p->ks = static_cast<int>(ks);
  p->cc = cc;
  p->xm = xm;
  p->nslot = static_cast<int>(nslot);
  p->nrows = 0;
  p->lds = static_cast<size_t>(kTC_OC * (cc * ks * ks + 1) + nslot * cc * Hp * Wp) * sizeof(float);
  return p->lds <= 64 * 1024;
}

constexpr int kPoolCB = 16;  // channels per workgroup of the pool pass (register window)

// One image addressed by a buffer descriptor with 32-bit byte offsets (the
// two register-window pool kernels); larger images take k_pad_lrn_maxpool.
inline bool pool_image_fits_rsrc(const fedagg_pool_args& a) {
  return a.C * a.H * a.W < (int64_t(1) << 29);
}

// Channels per LDS block of the sliding-window pool pass for this chain
// (k_pad_lrn_maxpool_slide, planes of <= 1024 positions, LRN size 0 / 3 /
// 4 / 5; <= 24 KiB of LDS), or 0 when the per-block kernels run it (or the
// caller asks for them with FEDAGG_POOL_PLANES).
int pool_slide_cb(const fedagg_pool_args& a, int64_t plane) {
  if (a.flags & FEDAGG_POOL_PLANES) return 0;
  if (!pool_image_fits_rsrc(a)) return 0;
  if (!(a.lrn_size == 0 || (a.lrn_size >= 3 && a.lrn_size <= 5))) return 0;
  const int64_t nq = (plane + 255) / 256;
  return nq == 1 ? 16 : nq <= 3 ? 8 : nq == 4 ? 4 : 0;
}

// ---------------------------------------------------------------------------
// The memory-bound chain that follows a convolution in the reference's CNNs
// (fedsim/models/simple_models.py:245-252, SimpleCNN2: relu -> F.pad(0,1,0,1)
// -> F.local_response_norm(size 4) -> F.max_pool2d(3, 2); SimpleCNN: relu ->
// max_pool2d(2, 2, padding 1)) as ONE pass: zero pad, LRN across channels,
// max pool.  A workgroup owns one image n and a block of CB channels: it
// builds the padded, normalised planes in LDS (each input element's LRN
// computed once, its channel window read from L1/L2) and max-pools them from
// there, so the conv output is read from HBM once and only the pooled output
// is written.  LRN follows torch.nn.functional.local_response_norm's ATen
// sequence: s = sum over the window of fl32(x*x) in channel order from +0,
// avg = s / size, d = pow(fl32(fl32(avg * alpha) + k), beta), y = x / d.
// Max pool: -inf start, NaN sticks (max_pool2d's CUDA kernel).
// ---------------------------------------------------------------------------
// LRN of one element from its channel window, ATen's sequence
// (torch/nn/functional.py local_response_norm): avg = s / size (exact as a
// multiply when size is a power of two), d = (avg * alpha + k) ^ beta, v / d.
// FAST: v * r with r = 1 / d = exp2(-beta * log2(b)) on the transcendental
// unit (v_log_f32 / v_exp_f32), no powf and no IEEE division (the pass is
// VALU-bound on them otherwise), within a few ulps of v / powf(b, beta);
// taken when b is a normal positive number and |beta * log2(b)| < 126 (r and
// 1 / r normal) -- the LRN's case, b >= k > 0.  Any other element
// (lrn_fast_scale false), and every element when !FAST, is v / powf(b, beta).
template <int SIZE>
__device__ __forceinline__ float lrn_base(float sum, float size_f, float alpha, float k) {
  float avg;
  if constexpr (SIZE > 0 && (SIZE & (SIZE - 1)) == 0)
    avg = sum * (1.0f / SIZE);
  else
    avg = sum / size_f;
  return avg * alpha + k;
}

__device__ __forceinline__ bool lrn_fast_scale(float b, float nbeta, float& r) {
  const float e = nbeta * __builtin_amdgcn_logf(b);
  r = __builtin_amdgcn_exp2f(e);
  return b >= 1.17549435e-38f && e > -126.0f && e < 126.0f;
}

// the rare powf of a fast LRN, out of line: the unrolled channel loops would
// otherwise carry one inlined powf each
__device__ __noinline__ float lrn_powf(float b, float beta) { return powf(b, beta); }

template <int SIZE, bool FAST>
__device__ __forceinline__ float lrn_value(float v, float sum, float size_f, float alpha,
                                           float beta, float k) {
  const float b = lrn_base<SIZE>(sum, size_f, alpha, k);
  if constexpr (FAST) {
    float r;
    return lrn_fast_scale(b, -beta, r) ? v * r : v / lrn_powf(b, beta);
  } else {
    return v / powf(b, beta);
  }
}

// Phase 2 of both variants: max-pool the CB padded planes in LDS into y.
__device__ __forceinline__ void pool_planes(const float* plane, int cbn, int Hp, int Wp,
                                            const fedagg_pool_args& a, int OH, int OW,
                                            float* __restrict__ yn) {
  const int OHW = OH * OW;
  const int HpWp = Hp * Wp;
  const int kh = static_cast<int>(a.pool_kh), kw = static_cast<int>(a.pool_kw);
  for (int e = threadIdx.x; e < cbn * OHW; e += 256) {
    const int cc = e / OHW;
    const int q = e - cc * OHW;
    const int oh = q / OW;
    const int ow = q - oh * OW;
    const int hs = oh * static_cast<int>(a.pool_sh) - static_cast<int>(a.pool_ph);
    const int ws = ow * static_cast<int>(a.pool_sw) - static_cast<int>(a.pool_pw);
    const int he = min(hs + kh, Hp), we = min(ws + kw, Wp);
    const int h0 = max(hs, 0), w0 = max(ws, 0);
    const float* pl = plane + cc * HpWp;
    float m = -__builtin_inff();
    for (int h = h0; h < he; ++h)
      for (int w = w0; w < we; ++w) {
        const float v = pl[h * Wp + w];
        if (v > m || __builtin_isnan(v)) m = v;
      }
    yn[e] = m;
  }
}

// pool_planes without a division per output: a thread's outputs e = t +
// 256 i advance their (channel, oh, ow) by the mixed-radix digits of 256;
// an unpadded 3 x 3 window (SimpleCNN2's pools) is read unrolled with no
// bounds.  The same selection as pool_planes: scan order h then w, a later
// element replaces the running max when greater or NaN.
__device__ __forceinline__ void pool_planes_step(const float* plane, int cbn, int Hp, int Wp,
                                                 const fedagg_pool_args& a, int OH, int OW,
                                                 float* __restrict__ yn) {
  const int OHW = OH * OW;
  const int HpWp = Hp * Wp;
  const int total = cbn * OHW;
  const int sh = static_cast<int>(a.pool_sh), sw = static_cast<int>(a.pool_sw);
  int e = threadIdx.x;
  int cc = e / OHW;
  int oh = (e - cc * OHW) / OW;
  int ow = e - cc * OHW - oh * OW;
  const int dcc = 256 / OHW;
  const int doh = (256 - dcc * OHW) / OW;
  const int dow = 256 - dcc * OHW - doh * OW;
  if (a.pool_kh == 3 && a.pool_kw == 3 && a.pool_ph == 0 && a.pool_pw == 0) {
    for (; e < total; e += 256) {
      const float* p = plane + cc * HpWp + oh * sh * Wp + ow * sw;
      float m = -__builtin_inff();
#pragma unroll
      for (int h = 0; h < 3; ++h)
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          const float v = p[h * Wp + w];
          if (v > m || __builtin_isnan(v)) m = v;
        }
      yn[e] = m;
      ow += dow;
      oh += doh;
      if (ow >= OW) { ow -= OW; ++oh; }
      cc += dcc;
      if (oh >= OH) { oh -= OH; ++cc; }
    }
    return;
  }
  const int kh = static_cast<int>(a.pool_kh), kw = static_cast<int>(a.pool_kw);
  for (; e < total; e += 256) {
    const int hs = oh * sh - static_cast<int>(a.pool_ph);
    const int ws = ow * sw - static_cast<int>(a.pool_pw);
    const int he = min(hs + kh, Hp), we = min(ws + kw, Wp);
    const int h0 = max(hs, 0), w0 = max(ws, 0);
    const float* pl = plane + cc * HpWp;
    float m = -__builtin_inff();
    for (int h = h0; h < he; ++h)
      for (int w = w0; w < we; ++w) {
        const float v = pl[h * Wp + w];
        if (v > m || __builtin_isnan(v)) m = v;
      }
    yn[e] = m;
    ow += dow;
    oh += doh;
    if (ow >= OW) { ow -= OW; ++oh; }
    cc += dcc;
    if (oh >= OH) { oh -= OH; ++cc; }
  }
}

// A K x K pool (K = 2, 3: the reference CNNs' pools) of one block with the
// window offsets mapped once per workgroup (src[i]: LDS index of the
// top-left member of output e = t + 256 i, the same for every block of the
// workgroup) over planes that carry the pool's padding as a -inf border (a
// -inf member is what max_pool2d's skipped padding is to the scan), and the
// max taken with v_maximum3_f32 (IEEE maximum: NaN-propagating, -0 < +0).
// That equals the scan-order rule of pool_planes_step (a later element
// replaces the running max when greater or NaN) unless the window holds a
// NaN (which NaN's bits) or a -0 (which zero's sign): the lanes whose window
// does -- the signed integer minimum of the members is INT_MIN exactly for a
// -0, the maximum is NaN for a NaN -- redo the scan.  3 x 3: four maximum3 +
// four min3_i32 per output instead of nine compare / NaN-test / select
// triples and the per-output index multiplies and bounds.
struct PoolStep {  // output e = t + 256 i of a block: its window, stepped
  int src, oh, ow;  // for i = 0: LDS index of the top-left member, its row, column
  int d_src, d_oh, d_ow;       // one step of 256 outputs in (channel, row, column) digits
  int wrap_ow_src, wrap_oh_src;  // src correction when a column / row digit wraps
  int OH, OW;
};

template <int K, int NI>
__device__ __forceinline__ void pool_mapped(const float* plane, const PoolStep& ps, int pitch,
                                            int total, float* __restrict__ yn) {
  constexpr int KK = K * K;
  int src = ps.src, oh = ps.oh, ow = ps.ow;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = static_cast<int>(threadIdx.x) + 256 * i;
    if (i > 0) {
      src += ps.d_src;
      oh += ps.d_oh;
      ow += ps.d_ow;
      if (ow >= ps.OW) {
        ow -= ps.OW;
        ++oh;
        src += ps.wrap_ow_src;
      }
      if (oh >= ps.OH) {
        oh -= ps.OH;
        src += ps.wrap_oh_src;
      }
    }
    if (e < total) {
      const float* p = plane + src;
      float v[KK];
#pragma unroll
      for (int h = 0; h < K; ++h)
#pragma unroll
        for (int w = 0; w < K; ++w) v[K * h + w] = p[h * pitch + w];
      float m = v[0];
      int mn = __builtin_bit_cast(int, v[0]);
#pragma unroll
      for (int t = 1; t < KK; ++t) {
        m = __builtin_elementwise_maximum(m, v[t]);
        mn = min(mn, __builtin_bit_cast(int, v[t]));
      }
      float r = m;
      if (mn == INT_MIN || m != m) {  // a -0 or a NaN in the window: the scan
        r = -__builtin_inff();
#pragma unroll
        for (int t = 0; t < KK; ++t)
          if (v[t] > r || __builtin_isnan(v[t])) r = v[t];
      }
      yn[e] = r;
    }
  }
}

// SIZE = the LRN window (0: no LRN) known at compile time: each thread loads
// the whole channel window of its pixel for the block (CB + SIZE - 1 values,
// all loads in flight at once) and normalises CB channels from registers.
// SIZE < 0: any window, loaded per channel (the general fallback).
template <int SIZE>
__global__ __launch_bounds__(256) void k_pad_lrn_maxpool(const float* __restrict__ x,
                                                         fedagg_pool_args a, int64_t CB,
                                                         int64_t OH, int64_t OW,
                                                         float* __restrict__ y) {
  extern __shared__ float plane[];
  const int64_t nblk = (a.C + CB - 1) / CB;
  const int64_t n = blockIdx.x / nblk;
  const int64_t c0 = (blockIdx.x - n * nblk) * CB;
  const int cbn = static_cast<int>(a.C - c0 < CB ? a.C - c0 : CB);
  const int H = static_cast<int>(a.H), W = static_cast<int>(a.W);
  const int Hp = H + static_cast<int>(a.pad_top + a.pad_bottom);
  const int Wp = W + static_cast<int>(a.pad_left + a.pad_right);
  const int HpWp = Hp * Wp;
  const int HW = H * W;
  const int C = static_cast<int>(a.C);
  const float* xn = x + n * a.C * HW;
  const float size_f = static_cast<float>(a.lrn_size);
  // the general path: every channel of the block for the pixel at plane
  // position q, its window loaded per channel, powf (any LRN size)
  auto general = [&](int q) {
    const int ph = q / Wp;
    const int ih = ph - static_cast<int>(a.pad_top);
    const int iw = q - ph * Wp - static_cast<int>(a.pad_left);
    const bool in = static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                    static_cast<unsigned>(iw) < static_cast<unsigned>(W);
    const int off = ih * W + iw;
    const int lo = static_cast<int>(a.lrn_size / 2);
    for (int cc = 0; cc < cbn; ++cc) {
      float v = 0.f;
      if (in) {
        const int c = static_cast<int>(c0) + cc;
        v = xn[c * HW + off];
        if (a.lrn_size > 0) {
          float sum = 0.f;
          for (int t = 0; t < a.lrn_size; ++t) {
            const int ch = c - lo + t;
            const float u =
                static_cast<unsigned>(ch) < static_cast<unsigned>(C) ? xn[ch * HW + off] : 0.f;
            sum = sum + u * u;
          }
          v = lrn_value<-1, false>(v, sum, size_f, a.lrn_alpha, a.lrn_beta, a.lrn_k);
        }
      }
      plane[cc * HpWp + q] = v;
    }
  };
  if constexpr (SIZE >= 0) {
    for (int q = threadIdx.x; q < HpWp; q += 256) {
      const int ph = q / Wp;
      const int ih = ph - static_cast<int>(a.pad_top);
      const int iw = q - ph * Wp - static_cast<int>(a.pad_left);
      const bool in = static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      const int off = ih * W + iw;
      constexpr int LO = SIZE / 2;
      constexpr int NV = kPoolCB + (SIZE > 0 ? SIZE - 1 : 0);
      float xr[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int ch = static_cast<int>(c0) - LO + j;
        xr[j] = (in && static_cast<unsigned>(ch) < static_cast<unsigned>(C) &&
                 ch < static_cast<int>(c0) + cbn + (SIZE > 0 ? SIZE - 1 - LO : 0))
                    ? xn[ch * HW + off] : 0.f;
      }
#pragma unroll
      for (int cc = 0; cc < kPoolCB; ++cc) {
        if (cc < cbn) {
          float v = xr[cc + LO];
          if constexpr (SIZE > 0) {
            float sum = 0.f;
#pragma unroll
            for (int t = 0; t < SIZE; ++t) sum = sum + xr[cc + t] * xr[cc + t];
            if (in) v = lrn_value<SIZE, true>(v, sum, size_f, a.lrn_alpha, a.lrn_beta, a.lrn_k);
          }
          plane[cc * HpWp + q] = v;
        }
      }
    }
  } else {
    for (int q = threadIdx.x; q < HpWp; q += 256) general(q);
  }
  __syncthreads();
  pool_planes(plane, cbn, Hp, Wp, a, static_cast<int>(OH), static_cast<int>(OW),
              y + (n * a.C + c0) * OH * OW);
}

// The same pass for planes of at most 256 * NQ positions (every pool of the
// reference's CNNs): grid (channel blocks, images) so the image's buffer
// descriptor is uniform, and ALL of a thread's NQ x (CB + SIZE - 1) channel
// window loads are issued before the first LRN, one latency per workgroup
// instead of one per 256 positions.  Per load: one VGPR offset for the
// position (out of range: past the descriptor, reads 0), the channel as the
// scalar offset.  Same arithmetic as k_pad_lrn_maxpool<SIZE>.
template <int SIZE, int NQ>
__global__ __launch_bounds__(256) void k_pad_lrn_maxpool_q(const float* __restrict__ x,
                                                           fedagg_pool_args a, int64_t CB,
                                                           int64_t OH, int64_t OW,
                                                           int64_t n_base,
                                                           float* __restrict__ y) {
  extern __shared__ float plane[];
  const int64_t n = n_base + blockIdx.y;
  const int c0 = static_cast<int>(blockIdx.x * CB);
  const int cbn = static_cast<int>(a.C - c0 < CB ? a.C - c0 : CB);
  const int H = static_cast<int>(a.H), W = static_cast<int>(a.W);
  const int Hp = H + static_cast<int>(a.pad_top + a.pad_bottom);
  const int Wp = W + static_cast<int>(a.pad_left + a.pad_right);
  const int HpWp = Hp * Wp;
  const int HW = H * W;
  const int C = static_cast<int>(a.C);
  const float* xn = x + n * a.C * HW;
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(xn), static_cast<short>(0), static_cast<int>(a.C * HW * 4), 0x00020000);
  constexpr uint32_t kOut = 0x80000000u;
  constexpr int LO = SIZE > 0 ? SIZE / 2 : 0;
  constexpr int NV = kPoolCB + (SIZE > 0 ? SIZE - 1 : 0);
  // the block's channels and their LRN halo: c0 - LO + j, j < NV, real
  // channels only (wave-uniform)
  const int jhi = cbn + (SIZE > 0 ? SIZE - 1 : 0);
  float xr[NQ][NV];
  uint32_t voff[NQ];
  bool in[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = threadIdx.x + 256 * i;
    const int ph = q / Wp;
    const int ih = ph - static_cast<int>(a.pad_top);
    const int iw = q - ph * Wp - static_cast<int>(a.pad_left);
    in[i] = q < HpWp && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
            static_cast<unsigned>(iw) < static_cast<unsigned>(W);
    voff[i] = in[i] ? static_cast<uint32_t>(ih * W + iw) * 4u : kOut;
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int ch = c0 - LO + j;
    const bool ok = ch >= 0 && ch < C && j < jhi;
#pragma unroll
    for (int i = 0; i < NQ; ++i)
      xr[i][j] = ok ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    xres, static_cast<int>(voff[i]), ch * HW * 4, 0))
                    : 0.f;
  }
  const float size_f = static_cast<float>(a.lrn_size);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < HpWp) {
#pragma unroll
      for (int cc = 0; cc < kPoolCB; ++cc) {
        if (cc < cbn) {
          float v = xr[i][cc + LO];
          if constexpr (SIZE > 0) {
            float sum = 0.f;
#pragma unroll
            for (int t = 0; t < SIZE; ++t) sum = sum + xr[i][cc + t] * xr[i][cc + t];
            if (in[i]) v = lrn_value<SIZE, true>(v, sum, size_f, a.lrn_alpha, a.lrn_beta, a.lrn_k);
          }
          plane[cc * HpWp + q] = v;
        }
      }
    }
  }
  __syncthreads();
  pool_planes(plane, cbn, Hp, Wp, a, static_cast<int>(OH), static_cast<int>(OW),
              y + (n * a.C + c0) * OH * OW);
}

// The same pass with the LRN channel window SLIDING in registers (planes of
// at most 256 * NQ positions).  A workgroup owns one image and a group of
// channels [g0, g1), walked in blocks of CB: each position's window
// (channels c - LO .. c + LEAD) lives in SW registers and advances one
// channel at a time, so every input element is read from HBM once (the
// per-block kernel above re-reads SIZE - 1 halo channels per block, across
// XCDs, and gets four workgroups per CU from 40 KiB planes; here the planes
// of a block take <= 20 KiB).  Software pipelined: the lead channels of
// block b + 1 are loaded while block b is pooled out of LDS.  Same
// arithmetic, element for element, as k_pad_lrn_maxpool_q<SIZE, NQ>.
template <int SIZE, int NQ, int CB>
__global__ __launch_bounds__(256) void k_pad_lrn_maxpool_slide(const float* __restrict__ x,
                                                               fedagg_pool_args a, int64_t CG,
                                                               int64_t OH, int64_t OW,
                                                               int64_t n_base,
                                                               float* __restrict__ y) {
  extern __shared__ float plane[];
  constexpr int LO = SIZE > 0 ? SIZE / 2 : 0;
  constexpr int SW = SIZE > 0 ? SIZE : 1;  // window registers per position
  constexpr int LEAD = SW - 1 - LO;         // channels the window reaches past c
  const int64_t n = n_base + blockIdx.y;
  const int C = static_cast<int>(a.C);
  const int g0 = static_cast<int>(blockIdx.x * CG);
  const int g1 = static_cast<int>(a.C - g0 < CG ? a.C : g0 + CG);
  const int H = static_cast<int>(a.H), W = static_cast<int>(a.W);
  const int Hp = H + static_cast<int>(a.pad_top + a.pad_bottom);
  const int Wp = W + static_cast<int>(a.pad_left + a.pad_right);
  const int HpWp = Hp * Wp;
  const int HW = H * W;
  const int OHW = static_cast<int>(OH * OW);
  const float* xn = x + n * a.C * HW;
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(xn), static_cast<short>(0), static_cast<int>(a.C * HW * 4), 0x00020000);
  constexpr uint32_t kOut = 0x80000000u;
  uint32_t voff[NQ];
  bool in[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = threadIdx.x + 256 * i;
    const int ph = q / Wp;
    const int ih = ph - static_cast<int>(a.pad_top);
    const int iw = q - ph * Wp - static_cast<int>(a.pad_left);
    in[i] = q < HpWp && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
            static_cast<unsigned>(iw) < static_cast<unsigned>(W);
    voff[i] = in[i] ? static_cast<uint32_t>(ih * W + iw) * 4u : kOut;
  }
  // 2 x 2 and 3 x 3 pools whose block fits NM outputs per thread (the
  // reference CNNs' pools: stride 2, a quarter of the plane's positions per
  // channel) take pool_mapped: the planes in LDS get the pool's padding as a
  // -inf border (pitch WpE, HpWpE per channel) and this thread's window
  // offsets are mapped once.  Other pools: pool_planes_step, no border.
  constexpr int NM = (CB * NQ + 3) / 4;
  const int pk = static_cast<int>(a.pool_kh);
  const bool map = a.pool_kh == a.pool_kw && (pk == 2 || pk == 3) && CB * OHW <= 256 * NM;
  const int bph = map ? static_cast<int>(a.pool_ph) : 0, bpw = map ? static_cast<int>(a.pool_pw) : 0;
  const int WpE = Wp + 2 * bpw;
  const int HpWpE = (Hp + 2 * bph) * WpE;
  PoolStep ps;
  {
    const int sh = static_cast<int>(a.pool_sh), sw = static_cast<int>(a.pool_sw);
    const int ow_n = static_cast<int>(OW), oh_n = static_cast<int>(OH);
    const int e = threadIdx.x;
    const int cc = e / OHW;
    ps.oh = (e - cc * OHW) / ow_n;
    ps.ow = e - cc * OHW - ps.oh * ow_n;
    ps.src = cc * HpWpE + ps.oh * sh * WpE + ps.ow * sw;
    const int dcc = 256 / OHW;
    ps.d_oh = (256 - dcc * OHW) / ow_n;
    ps.d_ow = 256 - dcc * OHW - ps.d_oh * ow_n;
    ps.d_src = dcc * HpWpE + ps.d_oh * sh * WpE + ps.d_ow * sw;
    ps.wrap_ow_src = sh * WpE - ow_n * sw;
    ps.wrap_oh_src = HpWpE - oh_n * sh * WpE;
    ps.OH = oh_n;
    ps.OW = ow_n;
  }
  // LDS index of each of this thread's plane positions inside the border
  int wq[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = threadIdx.x + 256 * i;
    const int ph = q / Wp;
    wq[i] = (ph + bph) * WpE + (q - ph * Wp) + bpw;
  }
  if (bph | bpw) {  // the border, once: the blocks write inside it only
    for (int e = threadIdx.x; e < CB * HpWpE; e += 256) plane[e] = -__builtin_inff();
    __syncthreads();
  }
  // channel ch of every position of this thread (0 outside [0, C): the
  // LRN's zero channels; padded positions read past the descriptor: 0)
  auto load = [&](float (&dst)[NQ], int ch) {
    const bool ok = ch >= 0 && ch < C;  // wave-uniform
#pragma unroll
    for (int i = 0; i < NQ; ++i)
      dst[i] = ok ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  xres, static_cast<int>(voff[i]), ch * HW * 4, 0))
                  : 0.f;
  };
  // The window of the current channel c: channel c - LO + t (t < SW) and its
  // square (each computed once).  RING (CB a multiple of SW, SimpleCNN2's
  // size-4 LRN): a ring whose slot for step j of a block is (j + t) % SW, a
  // compile-time index in the unrolled block, so nothing moves; else the
  // registers shift down one slot per channel.
  constexpr bool RING = CB % SW == 0;
  auto slot = [](int j, int t) { return RING ? (j + t) % SW : t; };
  float win[SW][NQ];
  float sq[SW][NQ];
#pragma unroll
  for (int t = 0; t + 1 < SW; ++t) {
    const int u = RING ? t : t + 1;  // the shifting form shifts them in before use
    load(win[u], g0 - LO + t);
#pragma unroll
    for (int i = 0; i < NQ; ++i) sq[u][i] = win[u][i] * win[u][i];
  }
  float raw[CB][NQ];  // the lead channels c + LEAD of the block in flight
#pragma unroll
  for (int j = 0; j < CB; ++j) load(raw[j], g0 + LEAD + j);
  const float size_f = static_cast<float>(a.lrn_size);
  const float nbeta = -a.lrn_beta;
  for (int c0 = g0; c0 < g1; c0 += CB) {
    const int cbn = g1 - c0 < CB ? g1 - c0 : CB;
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      if (j < cbn) {
        if constexpr (!RING) {
#pragma unroll
          for (int t = 0; t + 1 < SW; ++t)
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
              win[t][i] = win[t + 1][i];
              sq[t][i] = sq[t + 1][i];
            }
        }
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
          win[slot(j, SW - 1)][i] = raw[j][i];
          sq[slot(j, SW - 1)][i] = raw[j][i] * raw[j][i];
        }
        // lrn_value<SIZE, true> of every position without a per-lane branch:
        // the fast v * r everywhere, the powf division only when some lane
        // of the wave needs it (one wave-uniform branch per channel)
        float vv[NQ];
        float bb[NQ];
        bool slow = false;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
          vv[i] = win[slot(j, LO)][i];
          if constexpr (SIZE > 0) {
            // ATen's sum from +0 in channel order: a square is never -0,
            // so +0 + sq[0] is sq[0] and the chain starts there
            float sum = sq[slot(j, 0)][i];
#pragma unroll
            for (int t = 1; t < SIZE; ++t) sum = sum + sq[slot(j, t)][i];
            bb[i] = lrn_base<SIZE>(sum, size_f, a.lrn_alpha, a.lrn_k);
            float r;
            const bool fast = lrn_fast_scale(bb[i], nbeta, r);
            slow = slow || (in[i] && !fast);
            vv[i] = in[i] ? vv[i] * r : vv[i];
          }
        }
        if constexpr (SIZE > 0) {
          if (__builtin_expect(__ballot(slow) != 0, 0)) {
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
              float r;
              if (in[i] && !lrn_fast_scale(bb[i], nbeta, r))
                vv[i] = win[slot(j, LO)][i] / lrn_powf(bb[i], a.lrn_beta);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
          // positions 256 i + t of the first NQ - 1 groups are all inside
          if (i + 1 < NQ || static_cast<int>(threadIdx.x) + 256 * i < HpWp)
            plane[j * HpWpE + wq[i]] = vv[i];
        }
      }
    }
    // the next block's lead channels fly while this block is pooled
    if (c0 + CB < g1) {
#pragma unroll
      for (int j = 0; j < CB; ++j) load(raw[j], c0 + CB + LEAD + j);
    }
    __syncthreads();
    if (map && pk == 3)
      pool_mapped<3, NM>(plane, ps, WpE, cbn * OHW, y + (n * a.C + c0) * OHW);
    else if (map)
      pool_mapped<2, NM>(plane, ps, WpE, cbn * OHW, y + (n * a.C + c0) * OHW);
    else
      pool_planes_step(plane, cbn, Hp, Wp, a, static_cast<int>(OH), static_cast<int>(OW),
                       y + (n * a.C + c0) * OHW);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// The reference's arithmetic on bf16 / fp16 / fp64 client rows (the
// dtype-generic SerialAggregator keys: aggregators.py:17-40 on such
// tensors), and on fp32 rows held in separate allocations (RefF32 below:
// fedagg_reduce_rows_f32's wide-tile path).  ATen computes ``value * weight`` and ``sum_v + new_v`` of
// reduced-precision tensors in float (its opmath type) and rounds each result
// to the tensor's dtype; fp64 rounds each in double.  Per column, in arrival
// order:
//   s_1     = rnd(rnd(x_0 * w_0) + 0)         (the reference's 0 + tensor)
//   s_{k+1} = rnd(s_k + rnd(x_k * w_k))
// with w_k = the Python weight in the opmath type (fl32 for bf16 / fp16).
// No FMA (-ffp-contract=off): every product and sum rounds on its own.
// ---------------------------------------------------------------------------
// up: a stored element in the opmath type; rnd: an opmath value rounded to
// the dtype, kept in the opmath type; store_one: the dtype's bits of an already
// rounded value, a NaN as c10's scalar conversion writes it.  A NaN anywhere
// in a column's chain stays NaN to the end, so the hardware conversions (RNE,
// denormals kept) round every step and only the stored NaN is canonicalised.
// (NaN bits are not pinned by the reference: ATen's AVX-512 bf16 conversion
// writes 0xFFFF where its scalar one writes 0x7FC0.)
// The kernel's hooks, per 16-B (or narrower) vector of VW elements: the
// accumulator type ACC, first (s = rnd(rnd(x * w) + 0)), madd (s = rnd(s +
// rnd(x * w))), load (s from a stored running sum) and store.  RefEach spells
// them element by element from up / rnd / store_one.
template <class D, class T_, class OP_>
struct RefEach {
  using T = T_;
  using OP = OP_;
  using ACC = OP_;
  static constexpr bool kFinalize = false;  // divide by W32 before the store
  template <int VW> using V = T_ __attribute__((ext_vector_type(VW)));
  template <int VW>
  static __device__ __forceinline__ void first(OP_ (&s)[VW], const V<VW>& x, OP_ w) {
#pragma unroll
    for (int j = 0; j < VW; ++j) s[j] = D::rnd(D::rnd(D::up(x[j]) * w) + OP_(0));
  }
  template <int VW>
  static __device__ __forceinline__ void madd(OP_ (&s)[VW], const V<VW>& x, OP_ w) {
#pragma unroll
    for (int j = 0; j < VW; ++j) s[j] = D::rnd(s[j] + D::rnd(D::up(x[j]) * w));
  }
  template <int VW>
  static __device__ __forceinline__ void load(OP_ (&s)[VW], const V<VW>& a) {
#pragma unroll
    for (int j = 0; j < VW; ++j) s[j] = D::up(a[j]);
  }
  template <int VW>
  static __device__ __forceinline__ V<VW> store(const OP_ (&s)[VW]) {
    V<VW> o;
#pragma unroll
    for (int j = 0; j < VW; ++j) o[j] = D::store_one(s[j]);
    return o;
  }
};

struct RefBf16 : RefEach<RefBf16, uint16_t, float> {  // storage: the bf16 bits; opmath float
  static __device__ __forceinline__ float up(uint16_t u) {
    return __builtin_bit_cast(float, static_cast<uint32_t>(u) << 16);
  }
  static __device__ __forceinline__ float rnd(float x) {  // v_cvt_pk_bf16_f32
    return up(__builtin_bit_cast(uint16_t, static_cast<__bf16>(x)));
  }
  static __device__ __forceinline__ uint16_t store_one(float x) {  // c10::BFloat16: NaN -> 0x7FC0
    return x != x ? uint16_t(0x7FC0) : __builtin_bit_cast(uint16_t, static_cast<__bf16>(x));
  }
};

// fp16: the running sum stays in f16 registers and is added with v_pk_add_f16:
// for two f16 values fl16(fl32(s + p)) == fl16(s + p) (double rounding is
// innocuous for a sum when 24 >= 2 * 11 + 2; subnormal sums are exact in
// both), so the native add IS ATen's float-opmath add.  The product is not
// (w is an f32 weight): fl16(fl32(x * w)) keeps its two roundings -- the
// f32 products pass an empty register barrier before the conversion, else
// the compiler folds fptrunc(x * w) into v_fma_mixlo_f16, one rounding of
// the exact product, which differs on a tie of the first (3 of 8.4 M columns
// with w = 0.37, tests/test_generic_keys.py test_reference_kernel_tile_rungs).
struct RefF16 {  // storage: the fp16 bits; opmath float
  using T = uint16_t;
  using OP = float;
  using ACC = _Float16;
  static constexpr bool kFinalize = false;
  template <int VW> using V = uint16_t __attribute__((ext_vector_type(VW)));
  using f2 = float __attribute__((ext_vector_type(2)));
  using h2 = _Float16 __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ float up(uint16_t u) {
    return static_cast<float>(__builtin_bit_cast(_Float16, u));
  }
  template <int VW>
  static __device__ __forceinline__ void prod(_Float16 (&p)[VW], const V<VW>& x, float w) {
    if constexpr (VW % 2 == 0) {
#pragma unroll
      for (int j = 0; j < VW; j += 2) {
        f2 q = f2{up(x[j]), up(x[j + 1])} * w;  // v_pk_mul_f32
        asm("" : "+v"(q));
        const h2 r = __builtin_convertvector(q, h2);  // v_cvt_pk_f16_f32 (RNE)
        p[j] = r.x;
        p[j + 1] = r.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        float q = up(x[j]) * w;
        asm("" : "+v"(q));
        p[j] = static_cast<_Float16>(q);
      }
    }
  }
  template <int VW>
  static __device__ __forceinline__ void first(_Float16 (&s)[VW], const V<VW>& x, float w) {
    _Float16 p[VW];
    prod<VW>(p, x, w);
#pragma unroll
    for (int j = 0; j < VW; ++j) s[j] = p[j] + static_cast<_Float16>(0.f);  // -0 + 0 = +0
  }
  template <int VW>
  static __device__ __forceinline__ void madd(_Float16 (&s)[VW], const V<VW>& x, float w) {
    _Float16 p[VW];
    prod<VW>(p, x, w);
    if constexpr (VW % 2 == 0) {
#pragma unroll
      for (int j = 0; j < VW; j += 2) {
        const h2 r = h2{s[j], s[j + 1]} + h2{p[j], p[j + 1]};  // v_pk_add_f16
        s[j] = r.x;
        s[j + 1] = r.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < VW; ++j) s[j] = s[j] + p[j];
    }
  }
  template <int VW>
  static __device__ __forceinline__ void load(_Float16 (&s)[VW], const V<VW>& a) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      // through a scalar: __builtin_bit_cast of the vector element a[j] itself
      // read element 0 for every j (clang, ROCm 7.2)
      const uint16_t u = a[j];
      s[j] = __builtin_bit_cast(_Float16, u);
    }
  }
  template <int VW>
  static __device__ __forceinline__ V<VW> store(const _Float16 (&s)[VW]) {  // c10::Half: NaN -> sign | 0x7E00
    V<VW> o;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const uint16_t b = __builtin_bit_cast(uint16_t, s[j]);
      o[j] = s[j] != s[j] ? static_cast<uint16_t>((b & 0x8000u) | 0x7E00u) : b;
    }
    return o;
  }
};

struct RefF64 : RefEach<RefF64, double, double> {
  static __device__ __forceinline__ double up(double v) { return v; }
  static __device__ __forceinline__ double rnd(double v) { return v; }
  static __device__ __forceinline__ double store_one(double v) { return v; }
};

// fp32 client rows (fedagg_reduce_rows_f32's borrowed rows, round 5): the
// exact-mode sum acc = fl32(acc + fl32(x * w)) from +0, and FEDAGG_FINALIZE's
// IEEE division by fl32(W) -- the narrow kernel's arithmetic, bit for bit.
struct RefF32 : RefEach<RefF32, float, float> {
  static constexpr bool kFinalize = true;
  static __device__ __forceinline__ float up(float v) { return v; }
  static __device__ __forceinline__ float rnd(float v) { return v; }
  static __device__ __forceinline__ float store_one(float v) { return v; }
};

// One wave: a tile of NV * 64 consecutive VW-column vectors (a workgroup's
// four waves: four consecutive tiles), every row; one lane: NV vectors 64
// apart, so each load instruction reads 64 * VW consecutive elements of one
// row; U rows' loads in flight; columns from c_lo.  Row pointers and weights
// are wave-uniform.  Lanes past the last vector load the last one (in
// bounds) and store nothing.
template <class R, int VW, int U, int NV>
__global__ __launch_bounds__(256) void k_reduce_rows_ref(const typename R::T* const* __restrict__ rows,
                                                         const typename R::OP* __restrict__ w,
                                                         int64_t B, int64_t c_lo, int64_t P,
                                                         const typename R::T* __restrict__ acc_in,
                                                         typename R::T* __restrict__ out, int init,
                                                         typename R::OP W, int fin) {
  using T = typename R::T;
  using OP = typename R::OP;
  using ACC = typename R::ACC;
  using V = T __attribute__((ext_vector_type(VW)));
  using GV = const __attribute__((address_space(1))) V;  // global loads, not flat
  constexpr int kWaves = 256 / 64;
  const int64_t nvec = (P - c_lo) / VW;
  const int64_t ntiles = (nvec + 64 * NV - 1) / (64 * NV);
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWaves;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6); t < ntiles;
       t += nwaves) {
    int64_t c[NV];
    bool live[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int64_t i = t * (64 * NV) + v * 64 + lane;
      live[v] = i < nvec;
      c[v] = c_lo + (live[v] ? i : nvec - 1) * VW;
    }
    ACC s[NV][VW];
    int64_t k = 0;
    if (init) {
      const OP w0 = w[0];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const V x = *(GV*)(rows[0] + c[v]);
        R::template first<VW>(s[v], x, w0);
      }
      k = 1;
    } else {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const V a = *(GV*)(acc_in + c[v]);
        R::template load<VW>(s[v], a);
      }
    }
    for (; k + U <= B; k += U) {
      V x[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) x[u][v] = __builtin_nontemporal_load((GV*)(rows[k + u] + c[v]));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const OP wk = w[k + u];
#pragma unroll
        for (int v = 0; v < NV; ++v) R::template madd<VW>(s[v], x[u][v], wk);
      }
    }
    for (; k < B; ++k) {
      const OP wk = w[k];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const V x = __builtin_nontemporal_load((GV*)(rows[k] + c[v]));
        R::template madd<VW>(s[v], x, wk);
      }
    }
    if constexpr (R::kFinalize) {
      if (fin) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
          for (int j = 0; j < VW; ++j) s[v][j] = s[v][j] / W;
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (live[v]) *reinterpret_cast<V*>(out + c[v]) = R::template store<VW>(s[v]);
  }
}

// Workgroups: one per four tiles (the dispatcher balances them; past 2^30
// workgroups the waves stride over the rest).
inline int64_t rows_ref_blocks(int64_t nvec, int nv) {
  const int64_t tiles = (nvec + 64 * nv - 1) / (64 * nv);
  const int64_t g = (tiles + 3) / 4;
  return g < 1 ? 1 : (g < (int64_t(1) << 30) ? g : (int64_t(1) << 30));
}

template <class R, int VW, int U, int NV>
hipError_t launch_rows_ref_tile(const void* const* rows, const void* w, int64_t B, int64_t P,
                                const void* acc_in, void* out, bool init, int64_t body,
                                hipStream_t st, typename R::OP W = 0, bool fin = false) {
  using T = typename R::T;
  using OP = typename R::OP;
  auto rt = reinterpret_cast<const T* const*>(rows);
  auto wt = static_cast<const OP*>(w);
  auto ai = static_cast<const T*>(acc_in);
  auto ot = static_cast<T*>(out);
  if (body > 0)
    hipLaunchKernelGGL((k_reduce_rows_ref<R, VW, U, NV>), dim3(static_cast<uint32_t>(rows_ref_blocks(body / VW, NV))),
                       dim3(kBlock), 0, st, rt, wt, B, int64_t(0), body, ai, ot, init ? 1 : 0, W,
                       fin ? 1 : 0);
  if (body < P)  // columns past the last full vector (or every column: unaligned rows)
    hipLaunchKernelGGL((k_reduce_rows_ref<R, 1, U, NV>), dim3(static_cast<uint32_t>(rows_ref_blocks(P - body, NV))),
                       dim3(kBlock), 0, st, rt, wt, B, body, P, ai, ot, init ? 1 : 0, W,
                       fin ? 1 : 0);
  return hipGetLastError();
}

// Tile ladder, widest first.  A wave reading NV KiB of one row per load
// batch (16-B lanes) instead of 1 KiB keeps the K row streams' DRAM pages
// open longer: at K=200 x 50 MB rows the generic kernel went 5.6-5.9 ->
// 6.3-6.7 TB/s for U x NV = 2 x 8 (bf16), 4 x 8 (fp16) and 4 x 12 (fp64),
// bitwise the same sums (profiles/r05m*, r05n; bf16 at 4 x 8 spills).  A wide tile is taken only while the launch
// still has kRefMinBlocks workgroups (2 per CU): below that, the narrow tile
// (8 rows of 1 KiB in flight) fills the chip.
constexpr int64_t kRefMinBlocks = 512;

template <class R, int VW, int U, int NV>
hipError_t launch_rows_ref(const void* const* rows, const void* w, int64_t B, int64_t P,
                           const void* acc_in, void* out, bool init, bool vec, hipStream_t st) {
  const int64_t body = vec ? P / VW * VW : 0;
  const int64_t nvec = body ? body / VW : P;
  if (rows_ref_blocks(nvec, NV) >= kRefMinBlocks)
    return launch_rows_ref_tile<R, VW, U, NV>(rows, w, B, P, acc_in, out, init, body, st);
  if (rows_ref_blocks(nvec, 4) >= kRefMinBlocks)
    return launch_rows_ref_tile<R, VW, 4, 4>(rows, w, B, P, acc_in, out, init, body, st);
  return launch_rows_ref_tile<R, VW, 8, 1>(rows, w, B, P, acc_in, out, init, body, st);
}

// Which kernel fedagg_reduce_rows_f32 launches (host-side decision; the
// values are FEDAGG_ROWS_* of include/fedagg.h).  ``vec_ok``: out / acc_in
// are 16-B aligned and FEDAGG_SCALAR is clear; ``max_vw``: the most columns
// per lane P and the operands allow.
int rows_plan(int64_t P, int64_t B, int flags, bool vec_ok, int max_vw) {
  if (!row_fits_descriptor(P)) return FEDAGG_ROWS_FLAT;  // P = 2^30: flat loads
  if (fast_split(flags, P)) return FEDAGG_ROWS_SPLITK;
  // 16-B rows with no tuning field set: wide per-row tiles
  // (k_reduce_rows_ref<RefF32>, one wave = 8 or 4 KiB of each row per visit)
  // while the launch keeps kRefMinBlocks workgroups -- 6.0-6.1 -> 6.5-6.7
  // TB/s at 16-100 MB rows, bitwise the narrow kernel's sums (round 5,
  // profiles/r05p/, r05u/).  Any explicit tuning field (a forced mapping,
  // k-unroll, slots per lane or block size: an A/B caller asking for one
  // kernel) keeps the column kernels it names.
  constexpr int kTuningFields =
      FEDAGG_MAP_MASK | FEDAGG_UNROLL_MASK | FEDAGG_VPT_MASK | FEDAGG_BS_MASK;
  if (B > 0 && vec_ok && max_vw == 4 && (flags & kTuningFields) == 0) {
    if (rows_ref_blocks(P / 4, 8) >= kRefMinBlocks) return FEDAGG_ROWS_TILE4x8;
    if (rows_ref_blocks(P / 4, 4) >= kRefMinBlocks) return FEDAGG_ROWS_TILE8x4;
  }
  // misaligned rows take the one-column-per-lane kernel whatever the mapping
  const int vw = vec_ok ? narrow_vw(flags, P, B, max_vw) : 1;
  return vw ? FEDAGG_ROWS_NARROW1 + (vw == 2) + 2 * (vw == 4) : FEDAGG_ROWS_WIDE;
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

int fedagg_abi_version(void) { return FEDAGG_ABI_VERSION; }

int fedagg_column_mapping(int64_t P, int64_t B, int flags, int max_vw, int* vw, int* unroll) {
  if (P < 0 || B < 0 || !vw || !unroll || (max_vw != 1 && max_vw != 2 && max_vw != 4))
    return FEDAGG_EINVAL;
  *vw = narrow_vw(flags, P, B, max_vw);
  *unroll = *vw ? narrow_unroll(flags, P) : 0;
  return 0;
}

const char* fedagg_strerror(int code) {
  if (code == 0) return "success";
  if (code == FEDAGG_EINVAL) return "fedagg: invalid argument";
  if (code == FEDAGG_EALIGN) return "fedagg: misaligned pointer";
  if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
  return "fedagg: unknown error";
}

int fedagg_reduce_f32(const float* X, int64_t ldx, const float* w, int64_t B, int64_t P,
                      const float* acc_in, float* out, float W32, int flags, void* stream) {
  int rc = check_reduce_args(w, B, P, acc_in, out, flags);
  if (rc != 0 || P == 0) return rc;
  if (B > 0 && (!X || ldx < P)) return FEDAGG_EINVAL;
  const bool init = (flags & FEDAGG_INIT) != 0;
  const bool vec_ok = !(flags & FEDAGG_SCALAR) && aligned16(X) && (ldx % 4 == 0) &&
                      aligned16(out) && (init || aligned16(acc_in));
  // row k starts at X + k*ldx: ldx's alignment counts like a pointer's
  const int max_vw = (flags & FEDAGG_SCALAR)
                         ? 1
                         : max_cols_per_lane(P, {X, reinterpret_cast<const void*>(ldx * 4), out,
                                                 init ? nullptr : acc_in});
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (const int S = fast_split(flags, P))
    return static_cast<int>(launch_splitk(NarrowStrided{X, ldx}, S, w, B, P, acc_in,
                                          EpiStore{out}, W32, flags, s));
  // misaligned rows take the one-column-per-lane kernel whatever the mapping
  const int vw = vec_ok ? narrow_vw(flags, P, B, max_vw) : 1;
  if (vw) return static_cast<int>(launch_narrow_store(NarrowStrided{X, ldx}, vw, w, B, P, acc_in,
                                                      out, W32, flags, s));
  return static_cast<int>(dispatch_reduce(RowsStrided{X, ldx}, w, B, P, acc_in, out, W32, flags, s));
}

int fedagg_reduce_rows_f32(const float* const* rows, const float* w, int64_t B, int64_t P,
                           const float* acc_in, float* out, float W32, int flags,
                           void* stream) {
  int rc = check_reduce_args(w, B, P, acc_in, out, flags);
  if (rc != 0 || P == 0) return rc;
  if (B > 0 && !rows) return FEDAGG_EINVAL;
  // The table lives in device memory and cannot be inspected here without a
  // sync: the caller passes FEDAGG_SCALAR unless every rows[k] is 16-B aligned.
  const bool init = (flags & FEDAGG_INIT) != 0;
  const bool vec_ok = !(flags & FEDAGG_SCALAR) && aligned16(out) && (init || aligned16(acc_in));
  // without FEDAGG_SCALAR the caller promises 16-B aligned rows
  const int max_vw = (flags & FEDAGG_SCALAR)
                         ? 1
                         : max_cols_per_lane(P, {out, init ? nullptr : acc_in});
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool fin = (flags & FEDAGG_FINALIZE) != 0;
  const auto rt = reinterpret_cast<const void* const*>(rows);
  switch (rows_plan(P, B, flags, vec_ok, max_vw)) {
    case FEDAGG_ROWS_FLAT: {
      const EpiStore st{out};
      return static_cast<int>(
          (flags & FEDAGG_NT)
              ? launch_narrow_t<8, 1, true>(NarrowTableFlat{rows}, w, B, P, acc_in, st, W32, flags,
                                            s)
              : launch_narrow_t<8, 1, false>(NarrowTableFlat{rows}, w, B, P, acc_in, st, W32,
                                             flags, s));
    }
    case FEDAGG_ROWS_SPLITK:
      return static_cast<int>(launch_splitk(NarrowTable{rows, table_row_bytes(P)},
                                            fast_split(flags, P), w, B, P, acc_in, EpiStore{out},
                                            W32, flags, s));
    case FEDAGG_ROWS_TILE4x8:
      return static_cast<int>(
          launch_rows_ref_tile<RefF32, 4, 4, 8>(rt, w, B, P, acc_in, out, init, P, s, W32, fin));
    case FEDAGG_ROWS_TILE8x4:
      return static_cast<int>(
          launch_rows_ref_tile<RefF32, 4, 8, 4>(rt, w, B, P, acc_in, out, init, P, s, W32, fin));
    case FEDAGG_ROWS_WIDE:
      return static_cast<int>(dispatch_reduce(RowsTableBuf{rows, table_row_bytes(P)}, w, B, P,
                                              acc_in, out, W32, flags, s));
    default: {
      const int vw = vec_ok ? narrow_vw(flags, P, B, max_vw) : 1;
      return static_cast<int>(launch_narrow_store(NarrowTable{rows, table_row_bytes(P)}, vw, w, B,
                                                  P, acc_in, out, W32, flags, s));
    }
  }
}

int fedagg_rows_plan(int64_t P, int64_t B, int flags, int aligned16, int* kind) {
  if (P < 0 || B < 0 || !kind) return FEDAGG_EINVAL;
  const bool vec_ok = aligned16 && !(flags & FEDAGG_SCALAR);
  const int max_vw = (flags & FEDAGG_SCALAR) ? 1
                     : aligned16             ? max_cols_per_lane(P, {})
                                             : max_cols_per_lane(P, {reinterpret_cast<void*>(4)});
  *kind = rows_plan(P, B, flags, vec_ok, max_vw);
  return 0;
}

int fedagg_reduce_blocked_f32(const float* Xb, int64_t Kcap, int64_t C, const float* w,
                              int64_t B, int64_t P, const float* acc_in, float* out,
                              float W32, int flags, void* stream) {
  int rc = check_reduce_args(w, B, P, acc_in, out, flags);
  if (rc != 0 || P == 0) return rc;
  if (B > Kcap || (B > 0 && !Xb)) return FEDAGG_EINVAL;
  if (!valid_block_cols(C)) return FEDAGG_EINVAL;
  if (!aligned16(Xb) || !aligned16(out) || (!(flags & FEDAGG_INIT) && !aligned16(acc_in)))
    return FEDAGG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int bs_sel = (flags & FEDAGG_BS_MASK) >> FEDAGG_BS_SHIFT;
  if (bs_sel == 0) bs_sel = kDefaultBsSel;
  hipError_t e;
  const bool region32 = Kcap * C * 4 < (int64_t(1) << 32);
  const int vw = !region32 ? 0
                           : narrow_vw(flags, P, B,
                                       max_cols_per_lane(P, {out, (flags & FEDAGG_INIT) ? nullptr
                                                                                       : acc_in}));
  // buffer-descriptor path unless a block region is too large for a 32-bit
  // descriptor range (then flat loads)
  const int S = region32 ? fast_split(flags, P) : 0;
  if (S) {
    e = launch_splitk(NarrowBlocked{Xb, Kcap, C}, S, w, B, P, acc_in, EpiStore{out}, W32, flags,
                      s);
  } else if (vw) {
    e = launch_narrow_store(NarrowBlocked{Xb, Kcap, C}, vw, w, B, P, acc_in, out, W32, flags, s);
  } else if (!region32) {
    e = dispatch_blocked(RowsBlocked{Xb, Kcap, C}, C, bs_sel, w, B, P, acc_in, out, W32, flags, s);
  } else {
    e = dispatch_blocked(RowsBlockedBuf{Xb, Kcap, C}, C, bs_sel, w, B, P, acc_in, out, W32, flags,
                         s);
  }
  if (e == hipErrorInvalidValue) return FEDAGG_EINVAL;
  return static_cast<int>(e);
}

int fedagg_pack_segments_f32(const int64_t* segs, int64_t nseg, int64_t P, float* Xb,
                             int64_t Kcap, int64_t C, int64_t r, void* stream) {
  if (P < 0 || nseg < 0 || Kcap <= 0 || r < 0 || r >= Kcap) return FEDAGG_EINVAL;
  if (C != 1024 && C != 2048 && C != 4096) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!segs || nseg == 0 || !Xb || !aligned16(Xb)) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_pack_segments, dim3(pack_grid(P)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), segs, nseg, P, Xb, Kcap, C, r);
  return static_cast<int>(hipGetLastError());
}

int fedagg_unpack_row_f32(const float* Xb, int64_t Kcap, int64_t C, int64_t r, int64_t P,
                          float* dst, void* stream) {
  if (P < 0 || Kcap <= 0 || r < 0 || r >= Kcap) return FEDAGG_EINVAL;
  if (C != 1024 && C != 2048 && C != 4096) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!Xb || !dst || !aligned16(Xb) || !aligned16(dst)) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_unpack_row, dim3(elementwise_grid(P / 4 + 1)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), Xb, Kcap, C, r, P, dst);
  return static_cast<int>(hipGetLastError());
}

int fedagg_teacher_linear_f32(const float* x, int64_t x_kstride, const float* params,
                              int64_t params_kstride, int64_t w_off, int64_t b_off, int64_t K,
                              int64_t M, int64_t in, int64_t out, float* y, int flags,
                              void* stream) {
  if (K < 0 || M < 0 || in <= 0 || out <= 0 || x_kstride < 0 || params_kstride < 0 ||
      w_off < 0 || b_off < -1)
    return FEDAGG_EINVAL;
  if (flags & ~FEDAGG_RELU) return FEDAGG_EINVAL;
  // with several teachers, the layer must lie inside one teacher's vector
  if (K > 1 && (w_off + in * out > params_kstride || (b_off >= 0 && b_off + out > params_kstride)))
    return FEDAGG_EINVAL;
  if (K == 0 || M == 0) return 0;
  if (!x || !params || !y) return FEDAGG_EINVAL;
  const int64_t n_tiles = (out + kTL_N - 1) / kTL_N;
  const int64_t m_tiles = (M + kTL_M - 1) / kTL_M;
  // a 1-D grid: gridDim.x * blockDim.x must stay below 2^32, so the teachers
  // go in chunks of at most kMaxGridX / (tiles per teacher) per launch
  const int64_t per = n_tiles * m_tiles;
  const int64_t kMaxGridX = (int64_t(1) << 32) / 256 - 1;
  if (per > kMaxGridX) return FEDAGG_EINVAL;
  const int64_t kchunk = kMaxGridX / per;
  // the buffer-descriptor kernel: every teacher's rows 16-B aligned, the
  // per-teacher extents within 32-bit byte offsets
  const bool buf = (in % 4) == 0 && (x_kstride % 4) == 0 &&
                   (params_kstride % 4) == 0 && (w_off % 4) == 0 &&
                   (reinterpret_cast<uintptr_t>(x) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(params) % 16) == 0 && M * in < (int64_t(1) << 29) &&
                   out * in < (int64_t(1) << 29) && per < (int64_t(1) << 30);
  for (int64_t k0 = 0; k0 < K; k0 += kchunk) {
    const int64_t kn = K - k0 < kchunk ? K - k0 : kchunk;
    if (buf) {
      // wide layers stream each teacher's W once (weight-bound): at eight
      // workgroups per CU their 2048 concurrent row streams lose DRAM locality
      // (SimpleCNN's fc, in = 3136: 1049 vs 960 us for the generic kernel at
      // four per CU), so they reserve LDS for six per CU (round 4, warmed-up
      // interleaved A/B, profiles/r04w: SimpleCNN fc 0.927 -> 0.905 ms,
      // SimpleCNN2 fc1 0.523 -> 0.504 ms per 500 teachers against four; five
      // in between)
      const size_t pad = (in > kTL_WideIn) ? kTL_WidePadKB * 1024 : 0;
      hipLaunchKernelGGL(k_teacher_linear_buf, dim3(static_cast<unsigned>(kn * per)), dim3(256), pad,
                         static_cast<hipStream_t>(stream), x + k0 * x_kstride, x_kstride,
                         params + k0 * params_kstride, params_kstride, w_off, b_off,
                         static_cast<int>(M), static_cast<int>(in), static_cast<int>(out),
                         y + k0 * M * out, static_cast<int>(n_tiles), static_cast<int>(m_tiles),
                         (flags & FEDAGG_RELU) ? 1 : 0);
      const int rc = static_cast<int>(hipGetLastError());
      if (rc) return rc;
      continue;
    }
    hipLaunchKernelGGL(k_teacher_linear, dim3(static_cast<unsigned>(kn * per)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), x + k0 * x_kstride, x_kstride,
                       params + k0 * params_kstride, params_kstride, w_off, b_off, M, in, out,
                       y + k0 * M * out, n_tiles, m_tiles, (flags & FEDAGG_RELU) ? 1 : 0);
    const int rc = static_cast<int>(hipGetLastError());
    if (rc) return rc;
  }
  return 0;
}

int fedagg_conv_stage(int64_t R) {
  // reductions per LDS stage: 16 when that pads R less (conv1 of the reference's
  // CNNs: R = 3 * 5 * 5 = 75 -> 80 instead of 96), else 32
  if (R <= 0) return 0;
  return ((R + 15) / 16 * 16 < (R + 31) / 32 * 32) ? 16 : 32;
}

// 2 x 2 / stride 2 max pool padding requested by the conv flags, or -1
static int conv_pool_pad(int flags) {
  if (!(flags & FEDAGG_CONV_MAXPOOL2)) return -1;
  return (flags & FEDAGG_CONV_POOL_PAD1) ? 1 : 0;
}

int fedagg_conv_pool_fusable(const fedagg_conv2d_shape* shape, int flags) {
  if (!shape || !(flags & FEDAGG_CONV_MAXPOOL2) || (flags & FEDAGG_CONV_GATHER)) return 0;
  const fedagg_conv2d_shape& s = *shape;
  const int pp = conv_pool_pad(flags);
  if (s.OH + 2 * pp < 2 || s.OW + 2 * pp < 2 || s.M <= 0) return 0;
  const int64_t PH = (s.OH + 2 * pp - 2) / 2 + 1, PW = (s.OW + 2 * pp - 2) / 2 + 1;
  if (s.M * PH * PW * 4 >= (int64_t(1) << 31)) return 0;
  ConvLdsPlan plan;
  return conv_lds_plan(s, &plan, pp) && plan.cc == 0 ? 1 : 0;
}

int fedagg_conv_order(const fedagg_conv2d_shape* shape, int flags) {
  ConvLdsPlan plan;
  if (!shape || (flags & FEDAGG_CONV_GATHER) || !conv_lds_plan(*shape, &plan)) return 0;
  return plan.cc;
}

int fedagg_teacher_conv2d_f32(const float* x, int64_t x_kstride, const float* params,
                              int64_t params_kstride, int64_t w_off, int64_t b_off, int64_t K,
                              const fedagg_conv2d_shape* shape, float* y, int flags,
                              void* stream) {
  if (!shape || K < 0 || x_kstride < 0 || params_kstride < 0 || w_off < 0 || b_off < -1)
    return FEDAGG_EINVAL;
  if (flags & ~(FEDAGG_RELU | FEDAGG_CONV_GATHER | FEDAGG_CONV_MAXPOOL2 | FEDAGG_CONV_POOL_PAD1))
    return FEDAGG_EINVAL;
  if ((flags & FEDAGG_CONV_POOL_PAD1) && !(flags & FEDAGG_CONV_MAXPOOL2)) return FEDAGG_EINVAL;
  const int ppad = conv_pool_pad(flags);
  const fedagg_conv2d_shape s = *shape;
  const int64_t lim = int64_t(1) << 15;
  if (s.M < 0 || s.C <= 0 || s.H <= 0 || s.W <= 0 || s.OC <= 0 || s.KH <= 0 || s.KW <= 0 ||
      s.stride_h <= 0 || s.stride_w <= 0 || s.pad_h < 0 || s.pad_w < 0 || s.OH <= 0 || s.OW <= 0)
    return FEDAGG_EINVAL;
  if (s.H >= lim || s.W >= lim || s.KH >= lim || s.KW >= lim || s.stride_h >= lim ||
      s.stride_w >= lim || s.pad_h >= lim || s.pad_w >= lim || s.OH >= lim || s.OW >= lim ||
      s.H * s.W >= (int64_t(1) << 31))
    return FEDAGG_EINVAL;
  const int64_t R = s.C * s.KH * s.KW;
  if (K > 1 && (w_off + s.OC * R > params_kstride || (b_off >= 0 && b_off + s.OC > params_kstride)))
    return FEDAGG_EINVAL;
  // one teacher's input and weight matrix are addressed by 32-bit buffer offsets
  if (s.M * s.C * s.H * s.W >= (int64_t(1) << 29) || s.OC * R >= (int64_t(1) << 29))
    return FEDAGG_EINVAL;
  if (ppad >= 0 && !fedagg_conv_pool_fusable(&s, flags)) return FEDAGG_EINVAL;
  if (K == 0 || s.M == 0) return 0;
  if (!x || !params || !y) return FEDAGG_EINVAL;
  const int64_t oc_tiles = (s.OC + kTC_OC - 1) / kTC_OC;
  const int64_t px_tiles = (s.M * s.OH * s.OW + kTC_PX - 1) / kTC_PX;
  // gridDim.x * blockDim.x below 2^32 (256-lane tiles; the flat kernel's grid is no wider)
  if (px_tiles > (int64_t(1) << 32) / 256 - 1 || oc_tiles > 65535) return FEDAGG_EINVAL;
  const int relu = (flags & FEDAGG_RELU) ? 1 : 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  ConvLdsPlan plan;
  if (!(flags & FEDAGG_CONV_GATHER) && conv_lds_plan(s, &plan, ppad)) {
    // pixel slots per teacher (the pooled output's size when the pool is fused)
    const int64_t PHW = ppad >= 0 ? ((s.OH + 2 * ppad - 2) / 2 + 1) * ((s.OW + 2 * ppad - 2) / 2 + 1)
                                  : 0;
    const int64_t nslots = ppad >= 0 ? s.M * PHW * 4 : s.M * s.OH * s.OW;
    const int64_t y_kstride = ppad >= 0 ? s.M * s.OC * PHW : s.M * s.OC * s.OH * s.OW;
    for (int64_t k0 = 0; k0 < K; k0 += 65535) {
      const int64_t kn = K - k0 < 65535 ? K - k0 : 65535;
      const dim3 grid(static_cast<unsigned>(px_tiles), static_cast<unsigned>(oc_tiles),
                      static_cast<unsigned>(kn));
      const float* xk = x + k0 * x_kstride;
      const float* pk = params + k0 * params_kstride;
      float* yk = y + k0 * (ppad >= 0 ? y_kstride : s.M * s.OC * s.OH * s.OW);
#define FEDAGG_CONV_LDS(KS, CC, XM)                                                          \
  hipLaunchKernelGGL((k_teacher_conv2d_lds<KS, CC, XM>), grid, dim3(256), plan.lds, st, xk, \
                     x_kstride, pk, params_kstride, w_off, b_off, s, plan.nslot, yk, relu)
#define FEDAGG_CONV_LDS4(KS, CC, XM)                                                          \
  hipLaunchKernelGGL((k_teacher_conv2d_lds4<KS, CC, XM>), grid, dim3(256), plan.lds, st, xk, \
                     x_kstride, pk, params_kstride, w_off, b_off, s, plan.nslot, yk, relu)
#define FEDAGG_CONV_FLAT(KS, CI, XM)                                                          \
  do {                                                                                        \
    if (ppad >= 0) {                                                                          \
      if (half) FEDAGG_CONV_FLAT_H(KS, CI, XM, true, true);                                   \
      else FEDAGG_CONV_FLAT_H(KS, CI, XM, false, true);                                       \
    } else {                                                                                  \
      if (half) FEDAGG_CONV_FLAT_H(KS, CI, XM, true, false);                                  \
      else FEDAGG_CONV_FLAT_H(KS, CI, XM, false, false);                                      \
    }                                                                                         \
  } while (0)
#define FEDAGG_CONV_FLAT_H(KS, CI, XM, HF, PL)                                                \
  hipLaunchKernelGGL((k_teacher_conv2d_flat<KS, CI, XM, HF, PL>), gflat, dim3(kFlatThreads), plan.lds, st, xk, \
                     x_kstride, pk, params_kstride, w_off, b_off, s, plan.nslot, plan.nrows, yk, \
                     relu, ppad)
      if (plan.cc == 0) {
        const bool half = s.OC <= 32;
        const int64_t tpx = (half ? 2 : 1) * kFlatThreads;
        const dim3 gflat(static_cast<unsigned>((nslots + tpx - 1) / tpx),
                         static_cast<unsigned>(oc_tiles), static_cast<unsigned>(kn));
        if (plan.ks == 5) {
          if (s.C == 3) {
            if (plan.xm == 8) FEDAGG_CONV_FLAT(5, 3, 8); else FEDAGG_CONV_FLAT(5, 3, 16);
          } else {
            if (plan.xm == 8) FEDAGG_CONV_FLAT(5, 1, 8); else FEDAGG_CONV_FLAT(5, 1, 16);
          }
        } else {
          if (s.C == 3) {
            if (plan.xm == 8) FEDAGG_CONV_FLAT(3, 3, 8); else FEDAGG_CONV_FLAT(3, 3, 16);
          } else {
            if (plan.xm == 8) FEDAGG_CONV_FLAT(3, 1, 8); else FEDAGG_CONV_FLAT(3, 1, 16);
          }
        }
      } else if (plan.ks == 5) {  // chunks of 2 channels (conv_lds_plan)
        if (plan.xm == 8) FEDAGG_CONV_LDS4(5, 2, 8); else FEDAGG_CONV_LDS(5, 2, 16);
      } else {
        if (plan.xm == 8) FEDAGG_CONV_LDS4(3, 2, 8); else FEDAGG_CONV_LDS(3, 2, 16);
      }
#undef FEDAGG_CONV_FLAT
#undef FEDAGG_CONV_FLAT_H
#undef FEDAGG_CONV_LDS4
#undef FEDAGG_CONV_LDS
      const int rc = static_cast<int>(hipGetLastError());
      if (rc) return rc;
    }
    return 0;
  }
  for (int64_t k0 = 0; k0 < K; k0 += 65535) {  // grid z: at most 65535 teachers per launch
    const int64_t kn = K - k0 < 65535 ? K - k0 : 65535;
    const dim3 grid(static_cast<unsigned>(px_tiles), static_cast<unsigned>(oc_tiles),
                    static_cast<unsigned>(kn));
    const float* xk = x + k0 * x_kstride;
    const float* pk = params + k0 * params_kstride;
    float* yk = y + k0 * s.M * s.OC * s.OH * s.OW;
    if (fedagg_conv_stage(R) == 16)
      hipLaunchKernelGGL(k_teacher_conv2d<16>, grid, dim3(256), 0, st, xk, x_kstride, pk,
                         params_kstride, w_off, b_off, s, yk, relu);
    else
      hipLaunchKernelGGL(k_teacher_conv2d<32>, grid, dim3(256), 0, st, xk, x_kstride, pk,
                         params_kstride, w_off, b_off, s, yk, relu);
    const int rc = static_cast<int>(hipGetLastError());
    if (rc) return rc;
  }
  return static_cast<int>(hipGetLastError());
}

int fedagg_pool_output(const fedagg_pool_args* a, int64_t* OH, int64_t* OW, int64_t* CB) {
  if (!a || !OH || !OW || !CB) return FEDAGG_EINVAL;
  const int64_t lim = int64_t(1) << 15;
  if (a->N < 0 || a->C <= 0 || a->H <= 0 || a->W <= 0 || a->pad_top < 0 || a->pad_bottom < 0 ||
      a->pad_left < 0 || a->pad_right < 0 || a->lrn_size < 0 || a->lrn_size >= lim)
    return FEDAGG_EINVAL;
  const int64_t Hp = a->H + a->pad_top + a->pad_bottom, Wp = a->W + a->pad_left + a->pad_right;
  if (Hp >= lim || Wp >= lim || a->C >= (int64_t(1) << 30)) return FEDAGG_EINVAL;
  if (a->C * a->H * a->W >= (int64_t(1) << 31)) return FEDAGG_EINVAL;  // int offsets per image
  int64_t kh = a->pool_kh, kw = a->pool_kw, sh = a->pool_sh, sw = a->pool_sw;
  int64_t ph = a->pool_ph, pw = a->pool_pw;
  if (kh == 0) {  // no pooling: the padded, normalised planes themselves
    kh = kw = sh = sw = 1;
    ph = pw = 0;
  }
  if (kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || ph < 0 || pw < 0 || 2 * ph > kh || 2 * pw > kw ||
      kh >= lim || kw >= lim || sh >= lim || sw >= lim)
    return FEDAGG_EINVAL;
  if (Hp + 2 * ph < kh || Wp + 2 * pw < kw) return FEDAGG_EINVAL;
  *OH = (Hp + 2 * ph - kh) / sh + 1;
  *OW = (Wp + 2 * pw - kw) / sw + 1;
  const int64_t plane = Hp * Wp;
  if (plane > 16384) return FEDAGG_EINVAL;
  const int slide = pool_slide_cb(*a, plane);
  if (slide > 0) {  // sliding-window pass: channels per LDS block
    *CB = slide < a->C ? slide : a->C;
    return 0;
  }
  // channels per workgroup: at most kPoolCB, their padded planes within 40 KiB
  // of LDS (four workgroups per CU), balanced over the blocks
  int64_t cb = 10240 / plane;
  if (cb < 1) cb = 1;
  if (cb > kPoolCB) cb = kPoolCB;
  if (cb > a->C) cb = a->C;
  const int64_t nblk = (a->C + cb - 1) / cb;
  *CB = (a->C + nblk - 1) / nblk;
  return 0;
}

int fedagg_pad_lrn_maxpool_f32(const float* x, const fedagg_pool_args* args, float* y,
                               void* stream) {
  int64_t OH = 0, OW = 0, CB = 0;
  const int rc = fedagg_pool_output(args, &OH, &OW, &CB);
  if (rc) return rc;
  fedagg_pool_args a = *args;
  if (a.pool_kh == 0) {
    a.pool_kh = a.pool_kw = a.pool_sh = a.pool_sw = 1;
    a.pool_ph = a.pool_pw = 0;
  }
  if (a.N == 0) return 0;
  if (!x || !y) return FEDAGG_EINVAL;
  const int64_t blocks = a.N * ((a.C + CB - 1) / CB);
  if (blocks > (int64_t(1) << 31) - 1) return FEDAGG_EINVAL;
  const int64_t Hp = a.H + a.pad_top + a.pad_bottom, Wp = a.W + a.pad_left + a.pad_right;
  const size_t lds = static_cast<size_t>(CB * Hp * Wp) * sizeof(float);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nq = (Hp * Wp + 255) / 256;
  if (pool_slide_cb(a, Hp * Wp) > 0) {
    // channel groups: the whole C per image unless that leaves fewer than
    // 2048 workgroups; each group a multiple of the LDS block
    const int64_t cbs = pool_slide_cb(a, Hp * Wp);
    const int64_t nb = (a.C + cbs - 1) / cbs;
    int64_t G = (2048 + a.N - 1) / a.N;
    if (G > nb) G = nb;
    if (G < 1) G = 1;
    const int64_t CG = ((nb + G - 1) / G) * cbs;
    G = (a.C + CG - 1) / CG;
    // planes with the pool padding as a border (k_pad_lrn_maxpool_slide)
    const size_t slds = static_cast<size_t>(cbs * (Hp + 2 * a.pool_ph) * (Wp + 2 * a.pool_pw)) *
                        sizeof(float);
    for (int64_t n0 = 0; n0 < a.N; n0 += 65535) {
      const dim3 g(static_cast<unsigned>(G),
                   static_cast<unsigned>(a.N - n0 < 65535 ? a.N - n0 : 65535));
#define FEDAGG_POOL_S(SZ, Q, B)                                                                 \
  hipLaunchKernelGGL((k_pad_lrn_maxpool_slide<SZ, Q, B>), g, dim3(256), slds, st, x, a, CG, OH, \
                     OW, n0, y)
#define FEDAGG_POOL_SQ(SZ)                        \
  switch (nq) {                                   \
    case 1: FEDAGG_POOL_S(SZ, 1, 16); break;      \
    case 2: FEDAGG_POOL_S(SZ, 2, 8); break;       \
    case 3: FEDAGG_POOL_S(SZ, 3, 8); break;       \
    default: FEDAGG_POOL_S(SZ, 4, 4);             \
  }
      switch (a.lrn_size) {
        case 0: FEDAGG_POOL_SQ(0); break;
        case 3: FEDAGG_POOL_SQ(3); break;
        case 4: FEDAGG_POOL_SQ(4); break;
        default: FEDAGG_POOL_SQ(5);
      }
#undef FEDAGG_POOL_SQ
#undef FEDAGG_POOL_S
      const int rc = static_cast<int>(hipGetLastError());
      if (rc) return rc;
    }
    return 0;
  }
  if (nq <= 4 && (a.lrn_size == 0 || (a.lrn_size >= 3 && a.lrn_size <= 5)) &&
      pool_image_fits_rsrc(a)) {
    const int64_t nblk = (a.C + CB - 1) / CB;
    if (nblk > (int64_t(1) << 32) / 256 - 1) return FEDAGG_EINVAL;
    for (int64_t n0 = 0; n0 < a.N; n0 += 65535) {  // grid y: at most 65535 images per launch
      const dim3 g(static_cast<unsigned>(nblk),
                   static_cast<unsigned>(a.N - n0 < 65535 ? a.N - n0 : 65535));
#define FEDAGG_POOL_Q(SZ, Q)                                                                   \
  hipLaunchKernelGGL((k_pad_lrn_maxpool_q<SZ, Q>), g, dim3(256), lds, st, x, a, CB, OH, OW, n0, y)
#define FEDAGG_POOL_NQ(SZ)                              \
  switch (nq) {                                         \
    case 1: FEDAGG_POOL_Q(SZ, 1); break;                \
    case 2: FEDAGG_POOL_Q(SZ, 2); break;                \
    case 3: FEDAGG_POOL_Q(SZ, 3); break;                \
    default: FEDAGG_POOL_Q(SZ, 4);                      \
  }
      switch (a.lrn_size) {
        case 0: FEDAGG_POOL_NQ(0); break;
        case 3: FEDAGG_POOL_NQ(3); break;
        case 4: FEDAGG_POOL_NQ(4); break;
        default: FEDAGG_POOL_NQ(5);
      }
#undef FEDAGG_POOL_NQ
#undef FEDAGG_POOL_Q
      const int rc = static_cast<int>(hipGetLastError());
      if (rc) return rc;
    }
    return 0;
  }
  const dim3 grid(static_cast<unsigned>(blocks));
  switch (a.lrn_size) {
    case 0: hipLaunchKernelGGL(k_pad_lrn_maxpool<0>, grid, dim3(256), lds, st, x, a, CB, OH, OW, y); break;
    case 3: hipLaunchKernelGGL(k_pad_lrn_maxpool<3>, grid, dim3(256), lds, st, x, a, CB, OH, OW, y); break;
    case 4: hipLaunchKernelGGL(k_pad_lrn_maxpool<4>, grid, dim3(256), lds, st, x, a, CB, OH, OW, y); break;
    case 5: hipLaunchKernelGGL(k_pad_lrn_maxpool<5>, grid, dim3(256), lds, st, x, a, CB, OH, OW, y); break;
    default: hipLaunchKernelGGL(k_pad_lrn_maxpool<-1>, grid, dim3(256), lds, st, x, a, CB, OH, OW, y);
  }
  return static_cast<int>(hipGetLastError());
}

// Page-locked host memory (hipHostMalloc: torch's pin_memory) that the GPU
// reaches at the host address itself: kernels read and write it in place over
// PCIe -- 46-56 GB/s from 0.8 MB on, with no DMA to issue
// (tools/zero_copy_probe.hip, profiles/r06v/).
static bool host_mapped_here(const void* q) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, q) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not registered with HIP
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, const_cast<void*>(q), 0) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return dp == q;
}

int fedagg_host_mapped(const void* p, int64_t nbytes) {
  if (!p || nbytes < 0) return FEDAGG_EINVAL;
  const char* c = static_cast<const char*>(p);
  return host_mapped_here(c) && (nbytes == 0 || host_mapped_here(c + nbytes - 1)) ? 1 : 0;
}

int fedagg_pack_row_f32(const float* src, int64_t P, float* Xb, int64_t Kcap, int64_t C,
                        int64_t r, void* stream) {
  if (P < 0 || Kcap <= 0 || r < 0 || r >= Kcap) return FEDAGG_EINVAL;
  if (C != 1024 && C != 2048 && C != 4096) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!src || !Xb) return FEDAGG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipPointerAttribute_t attr;
  const bool known = hipPointerGetAttributes(&attr, src) == hipSuccess;
  (void)hipGetLastError();  // clear a failed query on pageable memory
  // HBM -> HBM, or page-locked host memory read in place over PCIe: the copy
  // kernel on the CUs; anything else (pageable, or mapped elsewhere) the DMA
  const float* from = nullptr;
  if (known && attr.type == hipMemoryTypeDevice)
    from = src;
  else if (known && attr.type == hipMemoryTypeHost &&
           fedagg_host_mapped(src, 4 * P) == 1)
    from = src;
  if (from && aligned16(from) && aligned16(Xb)) {
    hipLaunchKernelGGL(k_pack_row, dim3(pack_grid(P)), dim3(kBlock), 0, s, from,
                       P, Xb, Kcap, C, r);
    return static_cast<int>(hipGetLastError());
  }
  const int64_t full = P / C;
  const int64_t rem = P - full * C;
  float* dst = Xb + r * C;
  // One 2-D DMA: `full` segments of C floats, source pitch C, destination
  // pitch Kcap*C (the next column block of the same row), then the remainder.
  if (full > 0) {
    hipError_t e = hipMemcpy2DAsync(dst, static_cast<size_t>(Kcap * C) * 4, src,
                                    static_cast<size_t>(C) * 4, static_cast<size_t>(C) * 4,
                                    static_cast<size_t>(full), hipMemcpyDefault, s);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  if (rem > 0) {
    hipError_t e = hipMemcpyAsync(dst + full * Kcap * C, src + full * C,
                                  static_cast<size_t>(rem) * 4, hipMemcpyDefault, s);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return 0;
}

int fedagg_finalize_f32(const float* acc, float W32, int64_t P, float* out, void* stream) {
  if (P < 0) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!acc || !out || !aligned16(acc) || !aligned16(out)) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_finalize, dim3(elementwise_grid(P / 4 + 1)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), acc, W32, P, out);
  return static_cast<int>(hipGetLastError());
}

int fedagg_reduce_rows_ref(int dtype, const void* const* rows, const void* w, int64_t B,
                           int64_t P, const void* acc_in, void* out, int flags, void* stream) {
  const bool init = (flags & FEDAGG_INIT) != 0;
  if (dtype != FEDAGG_DTYPE_BF16 && dtype != FEDAGG_DTYPE_F16 && dtype != FEDAGG_DTYPE_F64)
    return FEDAGG_EINVAL;
  if (P < 0 || B < 0 || (init && B == 0)) return FEDAGG_EINVAL;
  if (flags & ~(FEDAGG_INIT | FEDAGG_SCALAR)) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!out || (!init && !acc_in) || (B > 0 && (!rows || !w))) return FEDAGG_EINVAL;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t es = dtype == FEDAGG_DTYPE_F64 ? 8 : 2;
  if (B == 0) {  // nothing to add: the running sum as it is
    if (out == acc_in) return 0;
    return static_cast<int>(hipMemcpyAsync(out, acc_in, P * es, hipMemcpyDeviceToDevice, st));
  }
  // 16-B vectors where the caller vouches for the rows (no FEDAGG_SCALAR) and
  // the accumulators are aligned too
  const bool vec = !(flags & FEDAGG_SCALAR) && aligned16(out) && (init || aligned16(acc_in));
  switch (dtype) {
    case FEDAGG_DTYPE_BF16:
      return static_cast<int>(launch_rows_ref<RefBf16, 8, 2, 8>(rows, w, B, P, acc_in, out, init, vec, st));
    case FEDAGG_DTYPE_F16:
      return static_cast<int>(launch_rows_ref<RefF16, 8, 4, 8>(rows, w, B, P, acc_in, out, init, vec, st));
    case FEDAGG_DTYPE_F64:
      return static_cast<int>(launch_rows_ref<RefF64, 2, 4, 12>(rows, w, B, P, acc_in, out, init, vec, st));
    default:
      return FEDAGG_EINVAL;
  }
}

int fedagg_finalize_f64(const double* acc, double W, int64_t P, double* out, void* stream) {
  if (P < 0) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!acc || !out || !aligned16(acc) || !aligned16(out)) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_finalize_f64, dim3(elementwise_grid(P / 2 + 1)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), acc, W, P, out);
  return static_cast<int>(hipGetLastError());
}

int fedagg_fedavg_sgd_f32(const float* avg, float lr, float* cloud, float* grad_out,
                          int64_t P, void* stream) {
  if (P < 0) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!avg || !cloud || !aligned16(avg) || !aligned16(cloud)) return FEDAGG_EINVAL;
  if (grad_out && !aligned16(grad_out)) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_fedavg_sgd, dim3(elementwise_grid(P / 4 + 1)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), avg, -lr, cloud, grad_out, P);
  return static_cast<int>(hipGetLastError());
}

int fedagg_adabest_sgd_f32(const float* avg, float beta, float lr, float* cloud,
                           float* avg_prev, float* grad_out, int64_t P, void* stream) {
  if (P < 0) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!avg || !cloud || !avg_prev) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_adabest_sgd, dim3(elementwise_grid(P)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), avg, beta, -lr, cloud, avg_prev,
                     grad_out, P);
  return static_cast<int>(hipGetLastError());
}

int fedagg_server_step_f32(int algo, const float* avg, float coef, float* cloud, float* aux,
                           float* avg_prev, float* momentum_buf, int momentum_init,
                           float* grad_out, const fedagg_sgd_params* sgd, int64_t P,
                           void* stream) {
  if (P < 0) return FEDAGG_EINVAL;
  StepPtrs sp;
  bool mom;
  int rc = make_step(algo, coef, cloud, aux, avg_prev, momentum_buf, momentum_init, grad_out,
                     nullptr, sgd, &sp, &mom);
  if (rc != 0) return rc;
  if (P == 0) return 0;
  if (!avg) return FEDAGG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = aligned16(avg) && step_aligned(sp);
  const dim3 g(elementwise_grid(vec ? P / 4 + 1 : P)), b(kBlock);
  hipError_t e = with_step(algo, mom, sp, [&](auto epi) {
    constexpr int A = decltype(epi)::kAlgo;
    constexpr bool M = decltype(epi)::kMom;
    if (vec)
      hipLaunchKernelGGL((k_server_step<A, M, true>), g, b, 0, s, avg, epi, P);
    else
      hipLaunchKernelGGL((k_server_step<A, M, false>), g, b, 0, s, avg, epi, P);
    return hipGetLastError();
  });
  if (e == hipErrorInvalidValue) return FEDAGG_EINVAL;
  return static_cast<int>(e);
}

int fedagg_reduce_step_blocked_f32(const float* Xb, int64_t Kcap, int64_t C, const float* w,
                                   int64_t B, int64_t P, const float* acc_in, float W32,
                                   int flags, const fedagg_step_args* step, void* stream) {
  if (!step) return FEDAGG_EINVAL;
  StepPtrs sp;
  bool mom;
  int rc = make_step(step->algo, step->coef, step->cloud, step->aux, step->avg_prev,
                     step->momentum_buf, step->momentum_init, step->grad_out, step->avg_out,
                     &step->sgd, &sp, &mom);
  if (rc != 0) return rc;
  rc = check_reduce_args(w, B, P, acc_in, step->cloud, flags);
  if (rc != 0 || P == 0) return rc;
  if (flags & FEDAGG_SCALAR) return FEDAGG_EINVAL;
  if (B > Kcap || (B > 0 && !Xb)) return FEDAGG_EINVAL;
  if (!valid_block_cols(C)) return FEDAGG_EINVAL;
  if (Kcap * C * 4 >= (int64_t(1) << 32)) return FEDAGG_EINVAL;
  if (!aligned16(Xb) || !step_aligned(sp) || (!(flags & FEDAGG_INIT) && !aligned16(acc_in)))
    return FEDAGG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const RowsBlockedBuf rows{Xb, Kcap, C};
  const int vw = narrow_vw(flags, P, B, max_cols_per_lane(P, {}));  // operands 16-B aligned
  // the per-C default configuration of fedagg_reduce_blocked_f32 (256 lanes,
  // VPT = C/1024, U = 4 at C=4096 else 2, non-temporal loads), or the narrow
  // mapping at small P
  const int S = fast_split(flags, P);
  hipError_t e = with_step(step->algo, mom, sp, [&](auto epi) {
    if (S) return launch_splitk(NarrowBlocked{Xb, Kcap, C}, S, w, B, P, acc_in, epi, W32, flags, s);
    if (vw)
      return launch_narrow_step(NarrowBlocked{Xb, Kcap, C}, vw, w, B, P, acc_in, epi, W32, flags,
                                s);
    switch (C) {
      case 4096: return launch_vec<256, 4, 4, true, RowsBlockedBuf>(rows, w, B, P, acc_in,
                                                                          epi, W32, flags, s);
      case 2048: return launch_vec<256, 2, 2, true, RowsBlockedBuf>(rows, w, B, P, acc_in,
                                                                          epi, W32, flags, s);
      case 1024: return launch_vec<256, 2, 1, true, RowsBlockedBuf>(rows, w, B, P, acc_in,
                                                                          epi, W32, flags, s);
      default: return hipErrorInvalidValue;
    }
  });
  if (e == hipErrorInvalidValue) return FEDAGG_EINVAL;
  return static_cast<int>(e);
}

int fedagg_reduce_step_rows_f32(const float* const* rows, const float* w, int64_t B,
                                int64_t P, const float* acc_in, float W32, int flags,
                                const fedagg_step_args* step, void* stream) {
  if (!step) return FEDAGG_EINVAL;
  StepPtrs sp;
  bool mom;
  int rc = make_step(step->algo, step->coef, step->cloud, step->aux, step->avg_prev,
                     step->momentum_buf, step->momentum_init, step->grad_out, step->avg_out,
                     &step->sgd, &sp, &mom);
  if (rc != 0) return rc;
  rc = check_reduce_args(w, B, P, acc_in, step->cloud, flags);
  if (rc != 0 || P == 0) return rc;
  if (flags & FEDAGG_SCALAR) return FEDAGG_EINVAL;
  if (B > 0 && !rows) return FEDAGG_EINVAL;
  if (!step_aligned(sp) || (!(flags & FEDAGG_INIT) && !aligned16(acc_in))) return FEDAGG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // the rows path's default configuration (256 lanes, kRowsVpt float4 slots
  // per lane, U = kRowsUnroll); the rows are the caller's separate
  // allocations, read through buffer descriptors
  const bool nt = (flags & FEDAGG_NT) != 0;
  if (!row_fits_descriptor(P)) {  // P = 2^30: flat loads, one column per lane
    hipError_t e = with_step(step->algo, mom, sp, [&](auto epi) {
      return launch_narrow_t<8, 1, true>(NarrowTableFlat{rows}, w, B, P, acc_in, epi, W32, flags,
                                         s);
    });
    if (e == hipErrorInvalidValue) return FEDAGG_EINVAL;
    return static_cast<int>(e);
  }
  const int vw = narrow_vw(flags, P, B, max_cols_per_lane(P, {}));  // operands 16-B aligned
  const int S = fast_split(flags, P);
  if (vw || S) {
    const NarrowTable tab{rows, table_row_bytes(P)};
    hipError_t e = with_step(step->algo, mom, sp, [&](auto epi) {
      if (S) return launch_splitk(tab, S, w, B, P, acc_in, epi, W32, flags, s);
      return launch_narrow_step(tab, vw, w, B, P, acc_in, epi, W32, flags, s);
    });
    if (e == hipErrorInvalidValue) return FEDAGG_EINVAL;
    return static_cast<int>(e);
  }
  auto go = [&](const auto& tab) {
    using T = std::decay_t<decltype(tab)>;
    return with_step(step->algo, mom, sp, [&](auto epi) {
      return nt ? launch_vec<kBlock, kRowsUnroll, kRowsVpt, true, T>(tab, w, B, P, acc_in,
                                                                          epi, W32, flags, s)
                : launch_vec<kBlock, kRowsUnroll, kRowsVpt, false, T>(
                      tab, w, B, P, acc_in, epi, W32, flags, s);
    });
  };
  hipError_t e = go(RowsTableBuf{rows, table_row_bytes(P)});
  if (e == hipErrorInvalidValue) return FEDAGG_EINVAL;
  return static_cast<int>(e);
}

int fedagg_feddyn_sgd_f32(const float* avg, float ratio, float lr, float* cloud, float* h,
                          float* avg_prev, float* grad_out, int64_t P, void* stream) {
  if (P < 0) return FEDAGG_EINVAL;
  if (P == 0) return 0;
  if (!avg || !cloud || !h) return FEDAGG_EINVAL;
  hipLaunchKernelGGL(k_feddyn_sgd, dim3(elementwise_grid(P)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), avg, ratio, -lr, cloud, h, avg_prev,
                     grad_out, P);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
