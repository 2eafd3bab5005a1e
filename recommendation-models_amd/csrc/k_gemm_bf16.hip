// k_gemm_bf16.hip -- bf16 instantiations of the tower GEMM (k_gemm.hpp with BF = true):
// v_mfma_f32_16x16x32_bf16, fp32 accumulation, bf16 weights / stored activations
// (BASELINE.json configs[4]: DCN and PNN with a bf16 table and bf16 weights).  A separate
// translation unit so the fp32 and bf16 kernel sets compile in parallel.
#include "k_gemm.hpp"

namespace rmx {

int launch_tower_bf16(hipStream_t s, GemmArgs& p, int nt, int amode, Epi epi) {
  switch (nt) {
#define RMX_NT(n) \
  case n: return launch_tower_nt<n, kPrecBF16>(s, p, amode, epi);
    RMX_NT(1) RMX_NT(2) RMX_NT(3) RMX_NT(4) RMX_NT(5) RMX_NT(6) RMX_NT(7)
    RMX_NT(8) RMX_NT(10) RMX_NT(13) RMX_NT(16) RMX_NT(20) RMX_NT(25) RMX_NT(26)
#undef RMX_NT
    default: set_error("bad tower width"); return RMX_E_INVALID;
  }
}

}  // namespace rmx

#if RMX_GEMM_DIAG & 8
// diagnostic builds only: the per-phase cycle sums of the last recorded bf16 GEMM launch (this
// translation unit's own copy of g_rmx_diag_t)
extern "C" int rmx_diag_phases_bf16(unsigned long long* out16) {
  return hipMemcpyFromSymbol(out16, HIP_SYMBOL(rmx::g_rmx_diag_t), sizeof(unsigned long long) * 18) == hipSuccess
             ? 0
             : -5;
}
#endif
