// Streaming-read microbenchmark: does the screens' per-lane row pattern
// (lane (r, h) of a wave reads 16-B pieces of row r at 128 h + 16 p: every
// wave-instruction touches 64 different 128-B lines) read X slower than a
// contiguous pattern (lane l reads bytes 16 l .. 16 l + 15 of a 1 KB span:
// 8 whole lines per instruction)?  Same bytes per wave, same occupancy, a
// sum kept live so nothing is dead-code eliminated.
//   hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o membench
//   ./membench [rows] [d]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                       \
    }                                                                \
  } while (0)

// one wave = 32 rows x (d doubles) per step; NP 16-B pieces per lane
template <int NP, int PAT, int PF>
__global__ void __launch_bounds__(256) k_read(const double *__restrict__ X,
                                              int64_t n, int d, double *out) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t step = (int64_t)gridDim.x * 4 * 32;
  const int rowb = d * 8;
  double acc = 0.0;
  double t[PF][NP * 2];
  auto load = [&](int slot, int64_t s0) {
    const int64_t rows = n - s0 > 0 ? n - s0 : 0;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(X + (s0 < n ? s0 : n) * d), 0,
        (int)(rows * rowb < 0x7fffffff ? rows * rowb : 0x7fffffff),
        0x00020000);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      uint32_t off;
      if (PAT == 0)  // row pattern: lane (r, h), piece p of its half row
        off = r * rowb + h * (rowb / 2) + 16 * p;
      else if (PAT == 1)  // contiguous: piece p = 1 KB span p of the tile
        off = 1024 * p + 16 * lane;
      else  // whole lines: K-step p / 4 (128 B per row), rows 8 (p % 4) + l / 8
        off = (8 * (p & 3) + (lane >> 3)) * rowb + 128 * (p >> 2) +
              16 * (lane & 7);
      const double2 v = __builtin_bit_cast(
          double2, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
      t[slot][2 * p] = v.x;
      t[slot][2 * p + 1] = v.y;
    }
  };
  int64_t s0 = wv * 32;
  if (PF > 1 && s0 < n) load(0, s0);
  for (; s0 < n; s0 += step) {
    if (PF == 1) load(0, s0);
    else if (s0 + step < n) load(1, s0 + step);
#pragma unroll
    for (int i = 0; i < NP * 2; ++i) acc += t[0][i];
    if (PF > 1) {
#pragma unroll
      for (int i = 0; i < NP * 2; ++i) t[0][i] = t[PF - 1][i];
    }
  }
  if (acc == 12345.678) out[0] = acc;
}

template <int NP, int PAT, int PF>
float run(const double *X, int64_t n, int d, double *out, int blocks) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_read<NP, PAT, PF><<<blocks, 256>>>(X, n, d, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int i = 0; i < reps; ++i) k_read<NP, PAT, PF><<<blocks, 256>>>(X, n, d, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
  const int d = argc > 2 ? atoi(argv[2]) : 32;
  double *X, *out;
  CK(hipMalloc(&X, n * d * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(X, 0, n * d * 8));
  const double gb = n * d * 8 / 1e9;
  for (int bpc : {2, 3, 4, 6, 8}) {
    const int blocks = 256 * bpc;
    if (d == 32) {
      float t0 = run<8, 0, 1>(X, n, d, out, blocks);
      float t1 = run<8, 1, 1>(X, n, d, out, blocks);
      float t2 = run<8, 0, 2>(X, n, d, out, blocks);
      float t3 = run<8, 2, 1>(X, n, d, out, blocks);
      printf("d=%d waves/CU=%2d  row %.3f ms %.0f GB/s | contig %.3f ms %.0f GB/s"
             " | row+pf %.3f ms %.0f GB/s | lines %.3f ms %.0f GB/s\n",
             d, bpc * 4, t0, gb / t0 * 1e3, t1, gb / t1 * 1e3, t2,
             gb / t2 * 1e3, t3, gb / t3 * 1e3);
    } else {
      float t0 = run<16, 0, 1>(X, n, d, out, blocks);
      float t1 = run<16, 1, 1>(X, n, d, out, blocks);
      float t2 = run<16, 2, 1>(X, n, d, out, blocks);
      printf("d=%d waves/CU=%2d  row %.3f ms %.0f GB/s | contig %.3f ms %.0f GB/s"
             " | lines %.3f ms %.0f GB/s\n",
             d, bpc * 4, t0, gb / t0 * 1e3, t1, gb / t1 * 1e3, t2,
             gb / t2 * 1e3);
    }
  }
  return 0;
}
