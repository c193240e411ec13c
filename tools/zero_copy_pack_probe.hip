// zero_copy_pack_probe.hip — how fast can a pack kernel read ONE client
// vector from page-locked host memory (the zero-copy host ingest,
// fedagg_pack_row_f32 on a mapped pointer)?  Variants of the slab-row copy
// (same destination layout: row r of a [ceil(P/C), Kcap, C] blocked slab),
// each timed with HIP events over many launches, one vector per launch:
//   tileU<U>_nt   the library's k_pack_row shape: a workgroup copies U*1024
//                 consecutive floats, U non-temporal 16-B loads per lane
//   tileU<U>      the same with ordinary loads
//   stride<G>     grid-stride loop over float4s, G workgroups
// Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -o tools/zero_copy_pack_probe tools/zero_copy_pack_probe.hip
//   ./tools/zero_copy_pack_probe P [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

using f32x4 = float __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

__device__ inline f32x4* dst_at(float* Xb, int64_t i, int64_t Kcap, int64_t C, int64_t r) {
  const int64_t cvec = C / 4;
  const int64_t b = i / cvec;
  return reinterpret_cast<f32x4*>(Xb + (b * Kcap + r) * C) + (i - b * cvec);
}

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void pack_tile(const float* __restrict__ src, int64_t P,
                                                     float* __restrict__ Xb, int64_t Kcap,
                                                     int64_t C, int64_t r) {
  constexpr int64_t kTile = int64_t(kBlock) * 4 * U;
  const int64_t nvec = P / 4;
  const int64_t ntiles = (P + kTile - 1) / kTile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = t * (kTile / 4) + int64_t(u) * kBlock + threadIdx.x;
      if (i < nvec)
        v[u] = NT ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src) + i)
                  : reinterpret_cast<const f32x4*>(src)[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = t * (kTile / 4) + int64_t(u) * kBlock + threadIdx.x;
      if (i < nvec) __builtin_nontemporal_store(v[u], dst_at(Xb, i, Kcap, C, r));
    }
  }
}

__global__ __launch_bounds__(kBlock) void pack_stride(const float* __restrict__ src, int64_t P,
                                                       float* __restrict__ Xb, int64_t Kcap,
                                                       int64_t C, int64_t r) {
  const int64_t nvec = P / 4;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nvec; i += stride)
    __builtin_nontemporal_store(reinterpret_cast<const f32x4*>(src)[i], dst_at(Xb, i, Kcap, C, r));
}

int main(int argc, char** argv) {
  const int64_t P = argc > 1 ? std::atoll(argv[1]) : 1085668;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 50;
  const int64_t C = 1024, Kcap = 4, r = 1;
  const int64_t Pv = P / 4 * 4;  // the tail is irrelevant to the timing
  const int64_t nblk = (Pv + C - 1) / C;
  float* h;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&h), Pv * 4, hipHostMallocDefault));
  for (int64_t i = 0; i < Pv; ++i) h[i] = 1e-3f * static_cast<float>(i % 9973);
  float* Xb;
  CHECK(hipMalloc(reinterpret_cast<void**>(&Xb), nblk * Kcap * C * 4));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> back(Pv);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CHECK(hipStreamSynchronize(s));
    std::vector<float> ts;
    for (int it = 0; it < reps; ++it) {
      CHECK(hipEventRecord(e0, s));
      launch();
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    // check the row: column p of row r sits at ((p / C) * Kcap + r) * C + p % C
    CHECK(hipMemset2DAsync(Xb + r * C, Kcap * C * 4, 0, C * 4, nblk, s));
    launch();
    for (int64_t b = 0; b < nblk; ++b) {
      const int64_t n = std::min<int64_t>(C, Pv - b * C);
      CHECK(hipMemcpyAsync(back.data() + b * C, Xb + (b * Kcap + r) * C, n * 4,
                           hipMemcpyDeviceToHost, s));
    }
    CHECK(hipStreamSynchronize(s));
    int64_t bad = 0;
    for (int64_t i = 0; i < Pv; ++i) bad += back[i] != h[i];
    const double us = ts[ts.size() / 2];
    std::printf("{\"variant\": \"%s\", \"P\": %lld, \"us\": %.1f, \"GBps\": %.1f, \"bad\": %lld}\n",
                name, static_cast<long long>(P), us, Pv * 4 / us * 1e-3,
                static_cast<long long>(bad));
    std::fflush(stdout);
  };
  auto tiles = [&](int U) { return static_cast<unsigned>((Pv + kBlock * 4 * U - 1) / (kBlock * 4 * U)); };
  run("tileU4_nt", [&] { hipLaunchKernelGGL((pack_tile<4, true>), dim3(tiles(4)), dim3(kBlock), 0, s, h, Pv, Xb, Kcap, C, r); });
  run("tileU4", [&] { hipLaunchKernelGGL((pack_tile<4, false>), dim3(tiles(4)), dim3(kBlock), 0, s, h, Pv, Xb, Kcap, C, r); });
  run("tileU1_nt", [&] { hipLaunchKernelGGL((pack_tile<1, true>), dim3(tiles(1)), dim3(kBlock), 0, s, h, Pv, Xb, Kcap, C, r); });
  run("tileU1", [&] { hipLaunchKernelGGL((pack_tile<1, false>), dim3(tiles(1)), dim3(kBlock), 0, s, h, Pv, Xb, Kcap, C, r); });
  run("tileU8", [&] { hipLaunchKernelGGL((pack_tile<8, false>), dim3(tiles(8)), dim3(kBlock), 0, s, h, Pv, Xb, Kcap, C, r); });
  for (int g : {256, 512, 1024, 2048})
    run(g == 256 ? "stride256" : g == 512 ? "stride512" : g == 1024 ? "stride1024" : "stride2048",
        [&] { hipLaunchKernelGGL(pack_stride, dim3(g), dim3(kBlock), 0, s, h, Pv, Xb, Kcap, C, r); });
  // the DMA path for comparison: H2D of the whole vector (into a scratch row region)
  float* d;
  CHECK(hipMalloc(reinterpret_cast<void**>(&d), Pv * 4));
  {
    for (int w = 0; w < 3; ++w) CHECK(hipMemcpyAsync(d, h, Pv * 4, hipMemcpyHostToDevice, s));
    CHECK(hipStreamSynchronize(s));
    std::vector<float> ts;
    for (int it = 0; it < reps; ++it) {
      CHECK(hipEventRecord(e0, s));
      CHECK(hipMemcpyAsync(d, h, Pv * 4, hipMemcpyHostToDevice, s));
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    std::printf("{\"variant\": \"dma_h2d\", \"P\": %lld, \"us\": %.1f, \"GBps\": %.1f}\n",
                static_cast<long long>(P), us, Pv * 4 / us * 1e-3);
  }
  return 0;
}
