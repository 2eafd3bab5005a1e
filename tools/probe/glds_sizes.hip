// Probe: where does a 1 / 2 / 4-byte global_load_lds put lane L's bytes in LDS?  Dumps the LDS
// image (0xEE prefill) after one wave-instruction per size.  Used to pick the w-ring layout.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int SZ>
__global__ void probe(const uint8_t* src, uint8_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xEE;
  __syncthreads();
  // lane L reads byte offset 4 * L + 1 (odd) for SZ = 1, 2 * L for SZ = 2 (16-bit aligned), 4 * L for SZ = 4
  const int lane = threadIdx.x;
  const uint8_t* s = src + (SZ == 1 ? 4 * lane + 1 : SZ * lane);
  auto* l = (__attribute__((address_space(3))) void*)lds;
  if constexpr (SZ == 1) __builtin_amdgcn_global_load_lds(s, l, 1, 0, 0);
  if constexpr (SZ == 2) __builtin_amdgcn_global_load_lds(s, l, 2, 0, 0);
  if constexpr (SZ == 4) __builtin_amdgcn_global_load_lds(s, l, 4, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}

int main() {
  uint8_t h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (uint8_t)i;
  uint8_t *d, *o;
  (void)hipMalloc(&d, 1024);
  (void)hipMalloc(&o, 1024);
  (void)hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
  uint8_t r[1024];
  hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, d, o);
  (void)hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
  printf("size1:");
  for (int i = 0; i < 24; ++i) printf(" %02x", r[i]);
  printf("\n");
  hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, d, o);
  (void)hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
  printf("size2:");
  for (int i = 0; i < 24; ++i) printf(" %02x", r[i]);
  printf(" ... [128..136]:");
  for (int i = 128; i < 136; ++i) printf(" %02x", r[i]);
  printf(" [252..260]:");
  for (int i = 252; i < 260; ++i) printf(" %02x", r[i]);
  printf("\n");
  hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, d, o);
  (void)hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
  printf("size4:");
  for (int i = 0; i < 24; ++i) printf(" %02x", r[i]);
  printf("\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
