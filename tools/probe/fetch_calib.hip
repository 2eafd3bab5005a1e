// Probe: what rocprofv3's FETCH_SIZE reports for the read widths the forward path uses
// (MI355X_MICROARCH.md §HBM: doubling is calibrated for 16-B-per-lane streaming reads only; "other
// access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Each kernel reads a known number of bytes from a 2 GiB buffer (past the 256 MiB Infinity Cache)
// and writes nothing (a never-true guard keeps the loads):
//   stream16      every byte once, 16 B per lane, coalesced
//   rows<R>       N distinct rows of R bytes (R = 4, 32, 64, 128) at scattered addresses
//                 (row i -> (i * P) mod nrows, P odd: a permutation), R / 16 lanes per row
//                 (R = 4: one lane, 4 B) -- the table-row gathers of the tower layer 1 (64 B fp32,
//                 32 B bf16), the first-order weights (4 B) and the sharded partition rows (128 B)
// Prints bytes / kernel time; the FETCH_SIZE pass (tools/fetch_calib.sh) gives reported / true bytes.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void stream16(const float4* __restrict__ src, int64_t n4, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = src[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}

template <int R>
__global__ void rows(const uint8_t* __restrict__ tab, int64_t nrows, int64_t n, int64_t P, float* out) {
  constexpr int LPR = R >= 16 ? R / 16 : 1;  // lanes per row
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t / LPR;
  const int part = (int)(t % LPR);
  if (i >= n) return;
  const int64_t row = (i * P) & (nrows - 1);  // nrows a power of two, P odd
  float s;
  if constexpr (R >= 16) {
    const float4 v = *reinterpret_cast<const float4*>(tab + row * R + part * 16);
    s = v.x + v.y + v.z + v.w;
  } else {
    s = *reinterpret_cast<const float*>(tab + row * R);
  }
  if (s == 1234.5f) out[0] = s;
}

int main() {
  const int64_t bytes = (int64_t)2 << 30;
  uint8_t* tab;
  float* out;
  if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(tab, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto timed = [&](const char* name, int64_t useful, auto&& launch) {
    launch();  // warm (TLB)
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-10s useful %8.1f MB  %8.3f ms  %7.1f GB/s\n", name, useful / 1e6, ms, useful / 1e6 / ms);
  };
  const int64_t n4 = bytes / 16;
  timed("stream16", bytes, [&] { hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const float4*)tab, n4, out); });
  const int64_t N = 2 << 20;  // rows gathered per launch
  const int64_t P = 2654435761LL;
#define RMX_ROWS(R)                                                                                              \
  {                                                                                                              \
    const int64_t nrows = bytes / R, lanes = N * (R >= 16 ? R / 16 : 1);                                        \
    timed("rows<" #R ">", N * R, [&] {                                                                           \
      hipLaunchKernelGGL(rows<R>, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, 0, tab, nrows, N, P, out); \
    });                                                                                                          \
  }
  RMX_ROWS(4) RMX_ROWS(32) RMX_ROWS(64) RMX_ROWS(128)
#undef RMX_ROWS
  (void)hipDeviceSynchronize();
  printf("N = %lld rows per gather launch; each kernel runs twice (warm + timed)\n", (long long)N);
  return 0;
}
