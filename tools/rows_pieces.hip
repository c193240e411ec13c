// Probe (not product code): does reading longer contiguous spans of each
// borrowed row per visit close the borrowed-rows vs column-blocked-slab gap
// (DESIGN §9 item 1, row-buffer locality hypothesis)?
//
// rows_pieces_f32(table, w, B, P, out, N, stream): one 64-lane wave owns N
// consecutive 512-byte pieces (N * 128 columns) of every row and visits the
// rows in order k = 0..B-1, reading its N pieces of row k back to back
// (N * 512 contiguous bytes per row visit), U = 4 rows of loads in flight.
// Same in-order fp32 arithmetic as the product kernel (a = fma-free a + x*w
// with -ffp-contract=off), so every N gives the same bits.
//
// slab_pieces_f32(X, Kcap, C, w, B, P, out, N, stream): the same wave shape
// over a column-blocked slab (element (k, p) at X[((p/C)*Kcap + k)*C + p%C]),
// N * 128 <= C, for a same-probe comparison.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC
//        -shared -o tools/librows_pieces.so tools/rows_pieces.hip
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

using f32x2 = float __attribute__((ext_vector_type(2)));
constexpr int kU = 4;

template <int N, class Addr>
__global__ __launch_bounds__(64) void k_pieces(Addr addr, const float* __restrict__ w, int64_t B,
                                               int64_t P, float* __restrict__ out) {
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * (128 * N) + threadIdx.x * 2;
  f32x2 a[N];
#pragma unroll
  for (int j = 0; j < N; ++j) a[j] = f32x2{0.f, 0.f};
  int64_t k = 0;
  for (; k + kU <= B; k += kU) {
    f32x2 v[kU][N];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const int64_t c = c0 + j * 128;
        v[u][j] = c < P ? __builtin_nontemporal_load(addr(k + u, c)) : f32x2{0.f, 0.f};
      }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const float wk = w[k + u];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        a[j].x = a[j].x + v[u][j].x * wk;
        a[j].y = a[j].y + v[u][j].y * wk;
      }
    }
  }
  for (; k < B; ++k) {
    const float wk = w[k];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int64_t c = c0 + j * 128;
      if (c < P) {
        const f32x2 x = __builtin_nontemporal_load(addr(k, c));
        a[j].x = a[j].x + x.x * wk;
        a[j].y = a[j].y + x.y * wk;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int64_t c = c0 + j * 128;
    if (c < P) *reinterpret_cast<f32x2*>(out + c) = a[j];
  }
}

struct TableAddr {
  const float* const* rows;
  __device__ __forceinline__ const f32x2* operator()(int64_t k, int64_t c) const {
    return reinterpret_cast<const f32x2*>(rows[k] + c);
  }
};

struct SlabAddr {
  const float* X;
  int64_t Kcap, C;
  __device__ __forceinline__ const f32x2* operator()(int64_t k, int64_t c) const {
    return reinterpret_cast<const f32x2*>(X + ((c / C) * Kcap + k) * C + c % C);
  }
};

template <class Addr>
int launch(int N, const Addr& addr, const float* w, int64_t B, int64_t P, float* out,
           hipStream_t s) {
  const int64_t span = 128 * static_cast<int64_t>(N);
  const dim3 grid(static_cast<unsigned>((P + span - 1) / span));
  switch (N) {
    case 1: k_pieces<1><<<grid, 64, 0, s>>>(addr, w, B, P, out); break;
    case 2: k_pieces<2><<<grid, 64, 0, s>>>(addr, w, B, P, out); break;
    case 4: k_pieces<4><<<grid, 64, 0, s>>>(addr, w, B, P, out); break;
    case 8: k_pieces<8><<<grid, 64, 0, s>>>(addr, w, B, P, out); break;
    case 16: k_pieces<16><<<grid, 64, 0, s>>>(addr, w, B, P, out); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
}

}  // namespace

extern "C" int rows_pieces_f32(const float* const* table, const float* w, int64_t B, int64_t P,
                               float* out, int N, void* stream) {
  if (P % 2) return -1;
  return launch(N, TableAddr{table}, w, B, P, out, static_cast<hipStream_t>(stream));
}

extern "C" int slab_pieces_f32(const float* X, int64_t Kcap, int64_t C, const float* w, int64_t B,
                               int64_t P, float* out, int N, void* stream) {
  if (P % 2 || C % (128 * N)) return -1;
  return launch(N, SlabAddr{X, Kcap, C}, w, B, P, out, static_cast<hipStream_t>(stream));
}
