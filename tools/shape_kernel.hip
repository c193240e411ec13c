// shape_kernel.hip — the microbenchmark reduce shape (tools/hbm_peak.hip
// reduce_pitch) exported with a C entry point, so tools/sweep_variants.py can
// run it on the SAME slab as libfedagg's kernel (same allocation, same data).
// Not exact-mode output (it keeps only a checksum); a measurement probe.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared \
//         -o tools/variants/libshape.so tools/shape_kernel.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

using f32x4 = float __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void reduce_shape(const f32x4* __restrict__ x, int K,
                                                   int64_t pitch, const float* __restrict__ w,
                                                   float* __restrict__ sink) {
  constexpr int ROW = 1024;
  const f32x4* base = x + static_cast<int64_t>(blockIdx.x) * pitch;
  f32x4 a[4] = {};
  int k = 0;
  for (; k + U <= K; k += U) {
    f32x4 v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[u][j] = __builtin_nontemporal_load(base + (k + u) * ROW + j * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wk = w[k + u];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = a[j] + v[u][j] * wk;
    }
  }
  const f32x4 t = a[0] + a[1] + a[2] + a[3];
  if (t.x + t.y + t.z + t.w == 12345.678f) sink[0] = 1.f;
}

extern "C" int shape_reduce(const float* Xb, int K, int64_t Kcap, int nblk, const float* w,
                            float* sink, void* stream) {
  hipLaunchKernelGGL(reduce_shape<4>, dim3(nblk), dim3(256), 0,
                     static_cast<hipStream_t>(stream), reinterpret_cast<const f32x4*>(Xb), K,
                     Kcap * 1024, w, sink);
  return static_cast<int>(hipGetLastError());
}
