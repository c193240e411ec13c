// wave_block.hip — does a smaller per-wave region beat the blocked reduce's
// 16 MiB per-workgroup region?  Same bytes (K rows x 6104*4096 columns, one
// allocation), read under different column-block widths C and thread
// mappings, exact-mode arithmetic (no FMA), timed interleaved in one process.
//
//   wg   C=4096: one 256-lane workgroup per block (the product kernel's shape:
//               4 waves share the block, each row is 16 KiB, VPT=4, U=4)
//   wave C=W:   one WAVE per block of W = 256*VPT columns (each row 1/2/4 KiB,
//               K rows contiguous => a K*W*4-byte region per wave), U rows of
//               loads in flight; 4 independent waves per workgroup
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/wave_block tools/wave_block.hip
//   ./tools/wave_block [K]
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#pragma clang fp contract(off)

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

using f32x4 = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 axpy4(f32x4 a, f32x4 x, float w) {
  a.x = a.x + x.x * w;
  a.y = a.y + x.y * w;
  a.z = a.z + x.z * w;
  a.w = a.w + x.w * w;
  return a;
}

// one 256-lane workgroup per C=4096 block (the product shape)
template <int U>
__global__ __launch_bounds__(256) void k_wg(const f32x4* __restrict__ x, int K,
                                          const float* __restrict__ w, f32x4* __restrict__ out) {
  constexpr int ROW = 1024;  // f32x4 slots per row of a block
  const f32x4* base = x + static_cast<int64_t>(blockIdx.x) * K * ROW;
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
      for (int j = 0; j < 4; ++j) a[j] = axpy4(a[j], v[u][j], wk);
    }
  }
  for (; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      a[j] = axpy4(a[j], __builtin_nontemporal_load(base + k * ROW + j * 256 + threadIdx.x), w[k]);
#pragma unroll
  for (int j = 0; j < 4; ++j) out[static_cast<int64_t>(blockIdx.x) * ROW + j * 256 + threadIdx.x] = a[j];
}

// one wave per block of 64*VPT slots; 4 waves (blocks) per workgroup
template <int VPT, int U>
__global__ __launch_bounds__(256) void k_wave(const f32x4* __restrict__ x, int K, int64_t nblk,
                                            const float* __restrict__ w, f32x4* __restrict__ out) {
  constexpr int ROW = 64 * VPT;
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (b >= nblk) return;
  const f32x4* base = x + b * K * ROW;
  f32x4 a[VPT] = {};
  int k = 0;
  for (; k + U <= K; k += U) {
    f32x4 v[U][VPT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        v[u][j] = __builtin_nontemporal_load(base + (k + u) * ROW + j * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wk = w[k + u];
#pragma unroll
      for (int j = 0; j < VPT; ++j) a[j] = axpy4(a[j], v[u][j], wk);
    }
  }
  for (; k < K; ++k)
#pragma unroll
    for (int j = 0; j < VPT; ++j)
      a[j] = axpy4(a[j], __builtin_nontemporal_load(base + k * ROW + j * 64 + lane), w[k]);
#pragma unroll
  for (int j = 0; j < VPT; ++j) out[b * ROW + j * 64 + lane] = a[j];
}

__global__ void fill(uint32_t* p, size_t n) {
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * 256) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ static_cast<uint32_t>(i >> 32);
    h ^= h >> 15;
    p[i] = 0x3c000000u | (h & 0x007fffffu);  // finite floats in [2^-7, 2^-6)
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 1000;
  const int64_t nblk4096 = 6104;
  const int64_t P = nblk4096 * 4096;
  const size_t bytes = static_cast<size_t>(K) * P * 4;
  f32x4* x;
  f32x4* out;
  float* w;
  CHECK(hipMalloc(&x, bytes));
  CHECK(hipMalloc(&out, P * 4));
  CHECK(hipMalloc(&w, K * 4));
  fill<<<8192, 256>>>(reinterpret_cast<uint32_t*>(x), bytes / 4);
  std::vector<float> hw(K);
  for (int k = 0; k < K; ++k) hw[k] = static_cast<float>(50 + (k * 37) % 551);
  CHECK(hipMemcpy(w, hw.data(), K * 4, hipMemcpyHostToDevice));
  CHECK(hipDeviceSynchronize());

  struct Var {
    const char* name;
    int C;
    int U;
  };
  auto launch = [&](int v) {
    switch (v) {
      case 0: k_wg<4><<<nblk4096, 256>>>(x, K, w, out); break;
      case 1: { const int64_t nb = P / 256;  k_wave<1, 16><<<(nb + 3) / 4, 256>>>(x, K, nb, w, out); } break;
      case 2: { const int64_t nb = P / 256;  k_wave<1, 8><<<(nb + 3) / 4, 256>>>(x, K, nb, w, out); } break;
      case 3: { const int64_t nb = P / 512;  k_wave<2, 8><<<(nb + 3) / 4, 256>>>(x, K, nb, w, out); } break;
      case 4: { const int64_t nb = P / 512;  k_wave<2, 4><<<(nb + 3) / 4, 256>>>(x, K, nb, w, out); } break;
      case 5: { const int64_t nb = P / 1024; k_wave<4, 4><<<(nb + 3) / 4, 256>>>(x, K, nb, w, out); } break;
      case 6: { const int64_t nb = P / 1024; k_wave<4, 2><<<(nb + 3) / 4, 256>>>(x, K, nb, w, out); } break;
    }
  };
  const Var vars[] = {{"wg C=4096 U=4", 4096, 4},  {"wave C=256 U=16", 256, 16},
                      {"wave C=256 U=8", 256, 8},  {"wave C=512 U=8", 512, 8},
                      {"wave C=512 U=4", 512, 4},  {"wave C=1024 U=4", 1024, 4},
                      {"wave C=1024 U=2", 1024, 2}};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  std::vector<std::vector<float>> ms(nv);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int v = 0; v < nv; ++v) launch(v);  // warm
  CHECK(hipDeviceSynchronize());
  for (int r = 0; r < 4; ++r) {
    for (int v = 0; v < nv; ++v) {
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < 3; ++i) launch(v);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / 3);
    }
  }
  CHECK(hipGetLastError());
  std::printf("[");
  for (int v = 0; v < nv; ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const double med = ms[v][ms[v].size() / 2];
    std::printf("%s{\"variant\": \"%s\", \"K\": %d, \"P\": %lld, \"ms_median\": %.4f, "
                "\"ms_min\": %.4f, \"GBps\": %.1f}",
                v ? ",\n " : "", vars[v].name, K, static_cast<long long>(P), med, ms[v][0],
                (static_cast<double>(bytes) + 4.0 * P) / med / 1e6);
  }
  std::printf("]\n");
  CHECK(hipFree(x));
  CHECK(hipFree(out));
  CHECK(hipFree(w));
  return 0;
}
