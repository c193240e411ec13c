// zero_copy_probe.hip — can the small host-resident rounds (BASELINE config 1:
// K=5 x 199 210 floats; config 2: K=10 x 1 085 668) skip the per-client DMA
// issue?  Measures, on page-locked host memory from hipHostMalloc (what
// torch's pin_memory hands out):
//   dma      hipMemcpyAsync H2D of K rows + stream sync (wall, and host issue
//            time per copy)
//   zc_read  one kernel reading the K host rows in place over PCIe (weighted
//            sum into HBM) + sync
//   zc_rw    the same kernel also writing its result to a host row
//   d2h      hipMemcpyAsync D2H of one row + sync
// and whether hipHostGetDevicePointer returns the host address itself.
// Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -o tools/zero_copy_probe tools/zero_copy_probe.hip
//   ./tools/zero_copy_probe K P [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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

struct Rows {
  const f32x4* r[16];
};

// out[i] = sum_k w_k * rows[k][i], float4 per lane, grid-stride
__global__ __launch_bounds__(256) void zc_sum(Rows rows, int K, size_t n4, f32x4* __restrict__ out,
                                              f32x4* __restrict__ host_out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) acc += rows.r[k][i] * (1.0f + k);
    out[i] = acc;
    if (host_out) host_out[i] = acc;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t P = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 199210;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 50;
  if (K < 1 || K > 16 || P < 4) {
    std::fprintf(stderr, "K in 1..16, P >= 4\n");
    return 2;
  }
  const size_t n4 = P / 4;  // the tail is irrelevant to the timing
  const size_t bytes = n4 * 16;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<float*> h(K + 1);
  for (int k = 0; k <= K; ++k) {
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&h[k]), bytes, hipHostMallocDefault));
    for (size_t i = 0; i < n4 * 4; ++i) h[k][i] = 1e-3f * static_cast<float>((i + k) % 977);
  }
  void* dp = nullptr;
  CHECK(hipHostGetDevicePointer(&dp, h[0], 0));
  hipPointerAttribute_t attr;
  CHECK(hipPointerGetAttributes(&attr, h[0]));
  std::vector<float*> d(K);
  for (int k = 0; k < K; ++k) CHECK(hipMalloc(reinterpret_cast<void**>(&d[k]), bytes));
  f32x4* out;
  CHECK(hipMalloc(reinterpret_cast<void**>(&out), bytes));
  Rows rows{};
  for (int k = 0; k < K; ++k) {
    void* p = nullptr;
    CHECK(hipHostGetDevicePointer(&p, h[k], 0));
    rows.r[k] = static_cast<const f32x4*>(p);
  }
  void* hout_dev = nullptr;
  CHECK(hipHostGetDevicePointer(&hout_dev, h[K], 0));
  const int grid = static_cast<int>(std::min<size_t>((n4 + 255) / 256, 2048));

  std::vector<double> t_dma, t_issue, t_zc, t_zcrw, t_d2h, t_kern;
  for (int it = 0; it < reps + 3; ++it) {
    double t0 = now_us();
    for (int k = 0; k < K; ++k) CHECK(hipMemcpyAsync(d[k], h[k], bytes, hipMemcpyHostToDevice, s));
    double t1 = now_us();
    CHECK(hipStreamSynchronize(s));
    double t2 = now_us();
    Rows drows{};
    for (int k = 0; k < K; ++k) drows.r[k] = reinterpret_cast<const f32x4*>(d[k]);
    double t3 = now_us();
    hipLaunchKernelGGL(zc_sum, dim3(grid), dim3(256), 0, s, drows, K, n4, out, nullptr);
    CHECK(hipStreamSynchronize(s));
    double t4 = now_us();
    hipLaunchKernelGGL(zc_sum, dim3(grid), dim3(256), 0, s, rows, K, n4, out, nullptr);
    CHECK(hipStreamSynchronize(s));
    double t5 = now_us();
    hipLaunchKernelGGL(zc_sum, dim3(grid), dim3(256), 0, s, rows, K, n4, out,
                       static_cast<f32x4*>(hout_dev));
    CHECK(hipStreamSynchronize(s));
    double t6 = now_us();
    CHECK(hipMemcpyAsync(h[K], out, bytes, hipMemcpyDeviceToHost, s));
    CHECK(hipStreamSynchronize(s));
    double t7 = now_us();
    if (it >= 3) {
      t_dma.push_back(t2 - t0);
      t_issue.push_back((t1 - t0) / K);
      t_kern.push_back(t4 - t3);
      t_zc.push_back(t5 - t4);
      t_zcrw.push_back(t6 - t5);
      t_d2h.push_back(t7 - t6);
    }
  }
  // the zero-copy result equals the DMA path's
  std::vector<float> a(n4 * 4);
  Rows drows{};
  for (int k = 0; k < K; ++k) drows.r[k] = reinterpret_cast<const f32x4*>(d[k]);
  hipLaunchKernelGGL(zc_sum, dim3(grid), dim3(256), 0, s, drows, K, n4, out, nullptr);
  CHECK(hipMemcpyAsync(a.data(), out, bytes, hipMemcpyDeviceToHost, s));
  CHECK(hipStreamSynchronize(s));
  hipLaunchKernelGGL(zc_sum, dim3(grid), dim3(256), 0, s, rows, K, n4, out,
                     static_cast<f32x4*>(hout_dev));
  CHECK(hipStreamSynchronize(s));
  size_t bad = 0;
  for (size_t i = 0; i < n4 * 4; ++i) bad += (a[i] != h[K][i]);
  const double mb = static_cast<double>(bytes) * K / 1e6;
  std::printf(
      "{\"K\": %d, \"P\": %zu, \"reps\": %d, \"device_ptr_is_host_ptr\": %s, \"attr_type\": %d, "
      "\"dma_us\": %.1f, \"dma_issue_us_per_copy\": %.2f, \"dma_GBps\": %.1f, "
      "\"kernel_hbm_us\": %.1f, \"zc_read_us\": %.1f, \"zc_read_GBps\": %.1f, "
      "\"zc_read_write_us\": %.1f, \"d2h_one_row_us\": %.1f, \"mismatches\": %zu}\n",
      K, P, reps, dp == h[0] ? "true" : "false", static_cast<int>(attr.type), median(t_dma),
      median(t_issue), mb / median(t_dma) * 1e3, median(t_kern), median(t_zc),
      mb / median(t_zc) * 1e3, median(t_zcrw), median(t_d2h), bad);
  return bad ? 1 : 0;
}
