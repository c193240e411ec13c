// pmc_calib.hip — calibrates rocprofv3's FETCH_SIZE for the load widths the
// reduce kernels use.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports
// half the bytes of a 16-B/lane streaming read, and other widths are
// uncalibrated.  Each kernel here reads a known 8 GiB (>> the 256 MiB
// Infinity Cache) exactly once with non-temporal buffer loads of one width —
// buffer_load_dword / _dwordx2 / _dwordx4, as k_reduce_narrow<VW=1>,
// k_reduce_narrow<VW=2> and k_reduce_vec issue them — so
//     factor(width) = 8 GiB / (FETCH_SIZE[KiB] * 1024)
// is the multiplier tools/pmc_traffic.py applies for that kernel.  The
// calib_write kernels do the same for WRITE_SIZE and 4 / 8 / 16-B stores.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o calib -- ./tools/pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr size_t kPiece = size_t(1) << 20;  // bytes per workgroup
constexpr int kU = 8;

// W dwords per lane per load; each workgroup streams its own 1 MiB piece.
template <int W>
__global__ __launch_bounds__(256) void calib_read(const char* buf, float* sink) {
  const char* piece = buf + static_cast<size_t>(blockIdx.x) * kPiece;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(piece), static_cast<short>(0), static_cast<int>(kPiece), 0x00020000);
  constexpr int kStep = 256 * W * 4;  // bytes per workgroup-wide load
  float acc = 0.f;
  for (int off = 0; off < static_cast<int>(kPiece); off += kU * kStep) {
    float v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int o = off + u * kStep + static_cast<int>(threadIdx.x) * W * 4;
      if constexpr (W == 1) {
        v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 2));
      } else if constexpr (W == 2) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 2);
        v[u] = __builtin_bit_cast(float, t[0]) + __builtin_bit_cast(float, t[1]);
      } else {
        const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 2);
        v[u] = __builtin_bit_cast(float, t[0]) + __builtin_bit_cast(float, t[1]) +
               __builtin_bit_cast(float, t[2]) + __builtin_bit_cast(float, t[3]);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) acc += v[u];
  }
  if (acc == 12345.678f) sink[0] = acc;  // keep the loads live
}

// W dwords per lane per store, each 1 MiB piece written once (WRITE_SIZE).
template <int W>
__global__ __launch_bounds__(256) void calib_write(char* buf) {
  char* piece = buf + static_cast<size_t>(blockIdx.x) * kPiece;
  constexpr int kStep = 256 * W * 4;
  for (int off = static_cast<int>(threadIdx.x) * W * 4; off < static_cast<int>(kPiece);
       off += kStep) {
    float* q = reinterpret_cast<float*>(piece + off);
#pragma unroll
    for (int e = 0; e < W; ++e) q[e] = 1.f;
  }
}

int main() {
  const size_t bytes = size_t(8) << 30;
  char* buf;
  float* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(buf, 0, bytes));
  const unsigned grid = static_cast<unsigned>(bytes / kPiece);
  for (int rep = 0; rep < 2; ++rep) {
    calib_read<1><<<grid, 256>>>(buf, sink);
    calib_read<2><<<grid, 256>>>(buf, sink);
    calib_read<4><<<grid, 256>>>(buf, sink);
    calib_write<1><<<grid, 256>>>(buf);
    calib_write<2><<<grid, 256>>>(buf);
    calib_write<4><<<grid, 256>>>(buf);
  }
  CHECK(hipDeviceSynchronize());
  CHECK(hipGetLastError());
  std::printf("{\"bytes_per_launch\": %zu}\n", bytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
