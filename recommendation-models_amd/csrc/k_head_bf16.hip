// k_head_bf16.hip -- bf16 tower layer 1 of DCN as a persistent row-owner kernel (gfx950), BASELINE.json
// configs[4].
//
// DCN's gathered layer 1 (model/encoder/HigherOrderEncoder.scala:34-59 over x = the gathered bf16 rows,
// ParRecModel.scala:279-306) with the cross stack's dot products as extra raw output columns
// (dcn/CrossEncoder.scala:40-55, the closed form of DESIGN.md §4: x0.w_l and x0.W_out[0:D] are columns
// N1 .. N1 + nx of the same GEMM) and the first order (bnn/Scatter.scala:17-36) fused in:
//   h1[m] = bf16(ReLU(x[m] W1^T + b1)) -> HBM (the bf16 tail's input, k_tail.hip)
//   xcol[m][j] = (x[m] W1^T)[N1 + j]    (cross_finish_kernel turns them into pre2)
//   fm_y[m] = y1                       (encoder_k16_kernel<0>'s sum, field order: bit-identical)
// Why: the column-sliced bf16 layer 1 (k_gemm.hpp, 64-row x 416 tiles) ran ~30 % above the random-line
// floor of its 2.56 M row gathers at 18 % MFMA busy: one 2-deep stage per block, so each
// block waits out its gathers.  Here a wave owns 16 samples and all 416 columns; its rows for step s + 2
// are gathered (from ids DMA'd a step earlier) while steps s and s + 1 compute, and the weights (one bf16
// plane, 26 KiB per K step) stream through the same kind of 3-slot LDS ring as k_rowown.hpp's.
// Per unit (= one 32-wide K step s) a wave issues, in this order: ids of step s + 3, rows + weights of
// step s + 2, 4 weight DMAs of step s + 2 -- 7 vector-memory instructions -- and waits at the unit start
// for all but the previous unit's last 6 (i.e. for its ids: the rows of step s + 2 need them).
#include "k_rowown.hpp"

namespace rmx {
namespace {
using namespace rowown;

constexpr int kBNT = 26;                      // column tiles computed: hidden columns + the cross columns
constexpr int kBUnit = kBNT * 1024;           // bytes per unit: 26 tiles x [16 rows][64 B] of one bf16 plane
constexpr int kBIns = kBUnit / 1024;          // 26 DMA instructions
constexpr int kBQ = (kBIns + kQW - 1) / kQW;  // 4 per wave (the last ones repeat instruction 25)
constexpr int kBSlots = 3;
constexpr int kBMaxF = 40;
constexpr int kBA = 4 * 1024;                 // per wave: 4 step slots x [2 fields][16 samples][32 B]
constexpr int kBId = 4 * 128;                 // per wave: 4 slots x [2 fields][16] ids
constexpr int kBWr = 4 * 128;                 // per wave: 4 slots x [2 fields][16] first-order weights (dwords)
constexpr int kBWave = kBA + kBId + kBWr;
constexpr size_t kBLds = (size_t)kBSlots * kBUnit + (size_t)kQW * kBWave + sizeof(float) * kQN;
static_assert(kBLds <= 160 * 1024, "LDS budget");
static_assert(kBQ == 4, "the static vmcnt counts below assume 4 weight DMAs per wave per unit");

struct HeadBArgs {
  int M, nblk, F, KS;
  const int32_t* ids;     // [M][F]
  const bf16_t* table;    // row of id at table + (id << gsh) (16 bf16: k = 16)
  int gsh;
  const bf16_t* wtab;     // first-order weight of id at wtab[id << wsh]
  int wsh;
  const bf16_t* W;        // [KS][416][32] bf16 (DenseLayer::W16)
  const float* b;         // [416]
  int N1;                 // hidden columns (ReLU, stored); columns [N1, N1 + nx) raw into xcol
  bf16_t* H;              // [M][416] out; columns >= N1 zero
  float* xcol;            // [M][xld] or null
  int nx, xld;
  float* fm_y;            // [M] y1 or null
};

__device__ __forceinline__ void b_wdma(const bf16_t* src, char* lds, int slot, int w, int q) {
  int ins = w + q * kQW;
  ins = ins < kBIns ? ins : kBIns - 1;
  int lo = (threadIdx.x & 63) >> 2;  // row of the tile; physical slot lane & 3 -> logical swz_slot(row, .)
  lo = lo * 32 + swz_slot(lo, threadIdx.x & 3) * 8;
  asm volatile("" : "+v"(lo));
  lds_dma<16>(src + ins * 16 * 32 + lo, lds + slot * kBUnit + ins * 1024);
}

// ids of K step c of row block rb into id slot `slot` (lanes 0 .. 31: field 2c + (L >> 4) of sample L & 15)
__device__ __forceinline__ void b_id_dma(const HeadBArgs& p, char* wl, int rb, int c, int slot, int w, int lane) {
  int f = lane >> 4, r = lane & 15;
  asm volatile("" : "+v"(f), "+v"(r));
  const int m = rb * kQBM + w * 16 + r, fld = 2 * c + f;
  const bool ok = rb < p.nblk && m < p.M && fld < p.F;
  const int32_t* src = ok ? p.ids + (int64_t)m * p.F + fld : g_rmx_neg1;
  if (lane < 32)
    lds_dma<4>(src, wl + kBA + slot * 128);
}

// rows of the wave's step s (one DMA: lane L = field L >> 5, sample (L >> 1) & 15, half L & 1 of the
// 32-B row) and its first-order weights (lanes 0 .. 31: a 2-byte DMA lands zero-extended in a dword)
__device__ __forceinline__ void b_row_dma(const HeadBArgs& p, char* wl, int s, int lane) {
  const int* ids = reinterpret_cast<const int*>(wl + kBA + (s & 3) * 128);
  int f = lane >> 5, r = (lane >> 1) & 15, hf = lane & 1, lw = lane & 31;
  asm volatile("" : "+v"(f), "+v"(r), "+v"(hf), "+v"(lw));
  const int id = ids[f * 16 + r], idw = ids[lw];
  const void* src = id >= 0 ? (const void*)(p.table + ((int64_t)id << p.gsh) + 8 * hf) : (const void*)g_rmx_zero16;
  const void* sw = idw >= 0 ? (const void*)(p.wtab + ((int64_t)idw << p.wsh)) : (const void*)g_rmx_zero16;
  lds_dma<16>(src, wl + (s & 3) * 1024);
  if (lane < 32)
    lds_dma<2>(sw, wl + kBA + kBId + (s & 3) * 128);
}

template <int N>
__device__ __forceinline__ void b_enter() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(kQThreads, 1) void tower_head_bf16_kernel(HeadBArgs p) {
  extern __shared__ __attribute__((aligned(16))) char bsmem[];
  char* lds = bsmem;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  char* wl = bsmem + kBSlots * kBUnit + w * kBWave;
  float* bl = reinterpret_cast<float*>(bsmem + kBSlots * kBUnit + kQW * kBWave);
  const int nit = (int)blockIdx.x < p.nblk ? (p.nblk - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int KS = p.KS;
  for (int i = tid; i < kQN; i += kQThreads) bl[i] = p.b ? p.b[i] : 0.f;
  const int fb = q_fbase(lane);

  // the wave's steps s = 0, 1, ... over its row blocks (step s: K step s % KS of row block
  // blockIdx.x + (s / KS) gridDim.x, none past the last); ring slots s & 3, weight-ring slot s % 3
  auto id_dma = [&](int s) {
    const int it = s / KS, c = s - it * KS;
    const int rb = it < nit ? (int)blockIdx.x + it * (int)gridDim.x : p.nblk;
    b_id_dma(p, wl, rb, c, s & 3, w, lane);
  };
  auto wsrc = [&](int s) { return p.W + (int64_t)(s % KS) * kQN * 32; };
  if (nit > 0) {
    for (int s = 0; s < 3; ++s) id_dma(s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int s = 0; s < 2; ++s) {
      b_row_dma(p, wl, s, lane);
#pragma unroll
      for (int q = 0; q < kBQ; ++q) b_wdma(wsrc(s), lds, s, w, q);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int slot = 0, s = 0;
  for (int it = 0; it < nit; ++it) {
    const int rb = blockIdx.x + it * gridDim.x;
    f32x4 acc[kBNT];
#pragma unroll
    for (int t = 0; t < kBNT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float y1 = 0.f;
#pragma unroll 1
    for (int c = 0; c < KS; ++c, ++s) {
      b_enter<6>();  // all but the previous unit's last 6 DMAs: its ids (for step s + 2) have landed
      int o = (g >> 1) * 512 + r16 * 32 + (g & 1) * 16;
      asm volatile("" : "+v"(o));
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(wl + (s & 3) * 1024 + o);
      {
        const uint32_t* wr = reinterpret_cast<const uint32_t*>(wl + kBA + kBId + (s & 3) * 128);
        y1 += __uint_as_float(wr[r16] << 16);  // first order, field order (encoder_k16_kernel<0>)
        y1 += __uint_as_float(wr[16 + r16] << 16);
      }
      id_dma(s + 3);
      b_row_dma(p, wl, s + 2, lane);
      __builtin_amdgcn_sched_barrier(0);
      const int ds = slot == 0 ? 2 : slot - 1;  // (slot + 2) mod 3
      const bf16_t* src = wsrc(s + 2);
      const char* ub = lds + slot * kBUnit;
      int fbu = fb;
      asm volatile("" : "+v"(fbu));
      constexpr int PF = 3;
      f32x4 bq[PF + 1];
#pragma unroll
      for (int t = 0; t < PF; ++t) bq[t] = *reinterpret_cast<const f32x4*>(ub + fbu + t * 1024);
#pragma unroll
      for (int t = 0; t < kBNT; ++t) {
        if (t + PF < kBNT) bq[(t + PF) % (PF + 1)] = *reinterpret_cast<const f32x4*>(ub + fbu + (t + PF) * 1024);
        if (t % 6 == 0 && t / 6 < kBQ) b_wdma(src, lds, ds, w, t / 6);
        __builtin_amdgcn_sched_barrier(0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bq[t % (PF + 1)]), a, acc[t], 0, 0, 0);
      }
      slot = slot == kBSlots - 1 ? 0 : slot + 1;
    }
    __builtin_amdgcn_sched_barrier(0);
    const int m = rb * kQBM + w * 16 + r16;
    int g4 = 4 * g;
    asm volatile("" : "+v"(g4));
    if (m < p.M) {
      bf16_t* hrow = p.H + (int64_t)m * kQN;
#pragma unroll
      for (int t = 0; t < kBNT; ++t) {
        const int n0 = 16 * t + g4;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + n0);
        f32x4 v = acc[t] + bb;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (n0 + r < p.N1 && v[r] > 0.f) ? v[r] : 0.f;
        *reinterpret_cast<bf16x4*>(hrow + n0) = __builtin_convertvector(v, bf16x4);
        if (p.xcol)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int e = n0 + r - p.N1;
            if (e >= 0 && e < p.nx) p.xcol[(int64_t)m * p.xld + e] = acc[t][r];
          }
      }
      if (g == 0 && p.fm_y) p.fm_y[m] = y1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool tower_head_bf16_usable(const DenseLayer& L1, int M, int F, int k, bool ids) {
  if (M <= 0 || !ids || k != 16 || F < 1 || F > kBMaxF || !L1.W16) return false;
  if (!(L1.K == 16 * F && L1.Npad == kQN && L1.N <= kQN && L1.bias_mode == 1 && L1.K1 < 0 &&
        L1.Kpad == (16 * F + 31) / 32 * 32))
    return false;
  // knob "bf16_head": 0 off, 2 always, 1 when the row blocks fill every CU at least once
  const int knob = tuning_get("bf16_head", 0);  // (default flipped on once measured on the GPU)
  if (knob == 0) return false;
  if (knob == 2) return true;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  return (M + kQBM - 1) / kQBM >= ncu;
}

int launch_tower_head_bf16(hipStream_t s, const DenseLayer& L1, int M, int F, const int32_t* ids, const bf16_t* table,
                           int ld, const bf16_t* wtab, int wld, bf16_t* H, int ldc, const XColArgs* xc, float* fm_y) {
  if (M <= 0) return RMX_OK;
  const int l = ld > 0 ? ld : 16, wl = wld > 0 ? wld : 1;
  if ((l & (l - 1)) || l < 16 || (wl & (wl - 1)) || ldc != kQN || !H || !L1.W16) {
    set_error("bf16 tower head: table / weight strides must be powers of two, h1 [M][416]");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipFuncSetAttribute((const void*)tower_head_bf16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kBLds));
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  HeadBArgs p{};
  p.M = M;
  p.nblk = (M + kQBM - 1) / kQBM;
  p.F = F;
  p.KS = (F + 1) / 2;
  p.ids = ids;
  p.table = table;
  p.gsh = __builtin_ctz((unsigned)l);
  p.wtab = wtab;
  p.wsh = __builtin_ctz((unsigned)wl);
  p.W = L1.W16;
  p.b = L1.b;
  p.N1 = L1.N1 >= 0 ? L1.N1 : L1.N;
  p.H = H;
  p.xcol = xc ? xc->ptr : nullptr;
  p.nx = xc ? xc->ld : 0;
  p.xld = xc ? xc->ld : 0;
  p.fm_y = fm_y;
  const int grid = std::min(p.nblk, std::max(ncu, 1));
  hipLaunchKernelGGL(tower_head_bf16_kernel, dim3(grid), dim3(kQThreads), kBLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
