// k_head_s3.hip -- fp32 tower layer 1 of DeepFM as a persistent row-owner kernel on the split GEMM (gfx950),
// BASELINE.json configs[1].
//
// Layer 1 of the tower (model/encoder/HigherOrderEncoder.scala:34-59: Linear(F k -> 400) + ReLU over
// x = Reshape(B, F k) of the gathered embeddings, ParRecModel.scala:279-306 makeEmbeddings), with the
// first order (bnn/Scatter.scala:17-36, the Scatter sum of the gathered weights) and the FM second order
// (SecondOrderEncoder.scala:19-34, the Mean over k of sum-square minus square-sum) fused in:
//   h1[m] = ReLU(x[m] W1^T + b1)  -> HBM (read once by the tail, k_tail_s3.hip)
//   fm_y[m] = y1 + 0.5 (sum_j (s_j^2 - q_j) / 16)   (encoder_k16_kernel<1>'s arithmetic: bit-identical)
// Why: the column-sliced split-GEMM layer 1 (k_gemm.hpp, 256 x 208 tiles) ran at ~0.44 of the split
// ceiling with ~50 % MFMA busy; the row-owner design of the tail (k_rowown.hpp: a wave owns 16 rows and
// all 416 columns, the weights stream through a 3-slot LDS ring, one barrier per unit) runs its layers
// at ~0.6.  Here the A operand is the gathered rows themselves: per K step (two fields) each wave DMAs
// its 16 samples' two 64-B rows into its own LDS slot, addressed by ids that were DMA'd into a small
// per-wave ring three steps earlier; the first-order weights ride a per-wave ring the same way.
//
// Per K step s (global across row blocks: row block s / KS, step s % KS) of a wave:
//   unit (c, half 0): wait, barrier; FM sums + first order + split of step s's rows; DMAs: ids of step
//                     s + 3, rows + weights of step s + 1 (from ids already in LDS), 5 weight-plane DMAs
//   unit (c, half 1): wait, barrier; 5 weight-plane DMAs
// so every unit's vector-memory count is static (9 / 5) and each wait is a compile-time vmcnt.
// LDS DMAs through the builtin in this translation unit (k_gemm.hpp lds_dma): measured faster here than
// the asm form, DeepFM 196.1-196.4 vs 193.4-194.0 M with the asm form (profiles/r04/ab_lds_dma_form.txt)
#define RMX_LDS_DMA_BUILTIN 1
#include "k_rowown.hpp"

namespace rmx {
namespace {
using namespace rowown;

constexpr int kHMaxF = 40;                       // fields (K = 16 F <= 640, 20 K steps)
constexpr int kHA = 2 * 2 * 16 * 64;             // per wave: 2 slots x [2 fields][16 samples][64 B]
constexpr int kHId = 4 * 128;                    // per wave: 4 slots x [2 fields][16] ids
constexpr int kHWr = 2 * 128;                    // per wave: 2 slots x [2 fields][16] first-order weights
constexpr int kHWave = kHA + kHId + kHWr;
constexpr size_t kHLds = (size_t)kQSlots * kQUnit + (size_t)kQW * kHWave + sizeof(float) * kQN;
static_assert(kHLds <= 160 * 1024, "LDS budget");

struct HeadS3Args {
  int M, F, KS;           // KS = ceil(F / 2) K steps
  QRows rows;             // full / half row blocks (k_rowown.hpp)
  const int32_t* ids;     // [M][F]
  const float* table;     // row of id at table + (id << gsh) (16 fp32: k = 16)
  int gsh;
  const float* wtab;      // first-order weight of id at wtab[id << wsh]
  int wsh;
  const bf16_t* W;        // [KS][3][416][32] split planes of Linear(16 F -> 400) (DenseLayer::W3)
  const float* b;         // [416]
  float* H;               // [M][416] out: ReLU(x W^T + b), columns 400 .. 415 zero
  float* fm_y;            // [M] y1 + y2 (fm_sums) or y1
  int fm_sums;
  float* X;               // XS (training forward): [M][ldx] the gathered rows x, as the encoder stores them
  int ldx;
  float* S;               // XS: [2][M][16] the FM sums s_j (field order), then the ReLU mask bits of h1 as
                          // uint32 (k_rowown.hpp bits_set; one pointer: a separate one spilled 179 SGPRs)
};

// XS: the x stores of rows past M / fields past F go here instead (every store is issued: the units'
// vector-memory counts stay static)
__device__ __attribute__((aligned(16))) float g_head_sink[64 * 4];

// K step c, half h of unit u (wave-uniform)
__device__ __forceinline__ const bf16_t* h_unit_src(const HeadS3Args& p, int u) {
  const int c = u >> 1, half = u & 1;
  return p.W + (int64_t)(c * 3 * kQN + half * kQUT * 16) * 32;
}

// ids of K step c of the row block at row0 (nw waves own rows) into id slot `slot` (lanes 0 .. 31: field
// 2c + (L >> 4) of sample L & 15; past M or F, or for a wave without rows: -1)
__device__ __forceinline__ void h_id_dma(const HeadS3Args& p, char* wl, int row0, int nw, int c, int slot, int w,
                                         int lane) {
  int f = lane >> 4, r = lane & 15;
  asm volatile("" : "+v"(f), "+v"(r));
  const int m = row0 + w * 16 + r, fld = 2 * c + f;
  const bool ok = w < nw && m < p.M && fld < p.F;
  const int32_t* src = ok ? p.ids + (int64_t)m * p.F + fld : g_rmx_neg1;
  if (lane < 32)
    lds_dma<4>(src, wl + kHA + slot * 128);
}

// rows (2 DMAs: field f = instruction, lane L: sample L >> 2, physical 16-B slot L & 3 = logical slot
// swz_slot(sample, L & 3)) and first-order weights (lanes 0 .. 31) of the wave's step s, from the ids
// in id slot s & 3, into A slot s & 1 / weight slot s & 1
__device__ __forceinline__ void h_row_dma(const HeadS3Args& p, char* wl, int s, int lane) {
  const int* ids = reinterpret_cast<const int*>(wl + kHA + (s & 3) * 128);
  int r = lane >> 2, g = swz_slot(lane >> 2, lane & 3), lw = lane & 31;
  asm volatile("" : "+v"(r), "+v"(g), "+v"(lw));
  const int id0 = ids[r], id1 = ids[16 + r], idw = ids[lw];
  const float* zero16 = g_rmx_zero16;
  const float* s0 = id0 >= 0 ? p.table + ((int64_t)id0 << p.gsh) + 4 * g : zero16;
  const float* s1 = id1 >= 0 ? p.table + ((int64_t)id1 << p.gsh) + 4 * g : zero16;
  const float* sw = idw >= 0 ? p.wtab + ((int64_t)idw << p.wsh) : zero16;
  char* a = wl + (s & 1) * 2048;
  lds_dma<16>(s0, a);
  lds_dma<16>(s1, a + 1024);
  if (lane < 32)
    lds_dma<4>(sw, wl + kHA + kHId + (s & 1) * 128);
}

// XS (training forward, k_head_s3 as DeepFM's layer 1 + encoder): also x and the FM sums, from the rows the
// head loads anyway -- two 16-B stores per half-0 unit (x of fields 2c, 2c + 1: a lane holds sample r16's
// j = 4g .. 4g + 3 of each) and one per row in the epilogue
template <bool XS>
__global__ __launch_bounds__(kQThreads, 1) void tower_head_s3_kernel(HeadS3Args p) {
  extern __shared__ __attribute__((aligned(16))) char hsmem[];
  char* lds = hsmem;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  char* wl = hsmem + kQSlots * kQUnit + w * kHWave;  // this wave's rows / ids / weights
  float* bl = reinterpret_cast<float*>(hsmem + kQSlots * kQUnit + kQW * kHWave);
  const int nit = p.rows.nit(blockIdx.x);
  const int KS = p.KS, NU = 2 * KS;  // units per row block

  for (int i = tid; i < kQN; i += kQThreads) bl[i] = p.b ? p.b[i] : 0.f;
  int lo = (lane >> 2) * 32 + swz_slot(lane >> 2, lane & 3) * 8;
  asm volatile("" : "+v"(lo));
  const int fb = q_fbase(lane);

  // the wave's steps s = 0, 1, ... run over its row blocks: step s is K step s % KS of row block
  // blockIdx.x + (s / KS) gridDim.x (none past the last); its ring slots are s & 3 (ids) and s & 1
  auto id_dma = [&](int s) {
    const int it = s / KS, c = s - it * KS;
    int row0, nw;
    p.rows.desc(blockIdx.x, it, row0, nw);
    h_id_dma(p, wl, row0, nw, c, s & 3, w, lane);
  };
  if (nit > 0) {
    for (int s = 0; s < 3; ++s) id_dma(s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    h_row_dma(p, wl, 0, lane);
    const bf16_t* s0 = h_unit_src(p, 0);
    const bf16_t* s1 = h_unit_src(p, 1);
#pragma unroll
    for (int qq = 0; qq < kQQ; ++qq) q_dma(s0, lds, 0, w, qq, lo);
#pragma unroll
    for (int qq = 0; qq < kQQ; ++qq) q_dma(s1, lds, 1, w, qq, lo);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int slot = 0, s = 0;
  for (int it = 0; it < nit; ++it) {
    int row0, nw;
    p.rows.desc(blockIdx.x, it, row0, nw);
    if (w >= nw) {
      // a half block's waves 4 .. 7: the same units, barriers and DMAs (ids of no rows), no MFMAs -- one
      // branch per row block (per-unit branches spilled the accumulators)
#pragma unroll 1
      for (int c = 0; c < KS; ++c, ++s) {
        q_enter<5>();
        id_dma(s + 3);
        h_row_dma(p, wl, s + 1, lane);
        __builtin_amdgcn_sched_barrier(0);
        const int u = 2 * c;
        int dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(h_unit_src(p, u + 2 < NU ? u + 2 : u + 2 - NU), lds, dslot, w, lo);
        slot = q_next(slot);
        q_enter<9>();
        dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(h_unit_src(p, u + 3 < NU ? u + 3 : u + 3 - NU), lds, dslot, w, lo);
        slot = q_next(slot);
      }
      continue;
    }
    f32x4 acc[kQNT];
#pragma unroll
    for (int t = 0; t < kQNT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 fs = f32x4{0.f, 0.f, 0.f, 0.f}, fq = fs;
    float y1 = 0.f;
#pragma unroll 1
    for (int c = 0; c < KS; ++c, ++s) {
      q_enter<5>();  // previous unit: (c - 1, half 1) or the previous row block's last, 5 DMAs
      bf16x8 ah, am, al;
      f32x4 xa0, xa1;  // (XS)
      {
        // rows of step s: a0 = field 2c, a1 = field 2c + 1 (zero past F), j = 4 g .. 4 g + 3
        int o = r16 * 64 + swz_slot(r16, g) * 16;
        asm volatile("" : "+v"(o));
        const char* a = wl + (s & 1) * 2048;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(a + o);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(a + 1024 + o);
        const float* wr = reinterpret_cast<const float*>(wl + kHA + kHId + (s & 1) * 128);
        {
#pragma clang fp contract(off)
          fm_accum(a0, a1, fs, fq);  // (SecondOrderEncoder sums, field order, k_gemm.hpp)
          y1 += wr[r16];             // first order in field order (encoder_k16_kernel<0>)
          y1 += wr[16 + r16];
        }
        split3(a0, a1, ah, am, al);
        xa0 = a0;
        xa1 = a1;
      }
      // ids three steps ahead (their slot held step s - 1's, read at step s - 2); rows + weights of the
      // next step into the A / weight slots step s - 1 used (its ids landed: issued at step s - 2)
      id_dma(s + 3);
      h_row_dma(p, wl, s + 1, lane);
      if constexpr (XS) {
        const int mx = row0 + w * 16 + r16, f0 = 2 * c;
        const bool okm = mx < p.M;
        float* sink = g_head_sink + lane * 4;
        float* xrow = p.X + (int64_t)mx * p.ldx + 4 * g;
        float* d0 = okm && f0 < p.F ? xrow + 16 * f0 : sink;
        float* d1 = okm && f0 + 1 < p.F ? xrow + 16 * (f0 + 1) : sink;
        *reinterpret_cast<f32x4*>(d0) = xa0;
        *reinterpret_cast<f32x4*>(d1) = xa1;
      }
      __builtin_amdgcn_sched_barrier(0);  // these 4 (XS: 6) ahead of the unit's 5 (the static vmcnt counts)
      const int u = 2 * c;
      int dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQUT, 0>(lds + slot * kQUnit, fb, ah, am, al, acc, h_unit_src(p, u + 2 < NU ? u + 2 : u + 2 - NU), lds,
                      dslot, w, lo);
      slot = q_next(slot);
      q_enter<XS ? 11 : 9>();  // previous unit: 1 id + 2 row + 1 weight (+ 2 x stores) + 5 plane DMAs
      dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQNT - kQUT, kQUT>(lds + slot * kQUnit, fb, ah, am, al, acc,
                                h_unit_src(p, u + 3 < NU ? u + 3 : u + 3 - NU), lds, dslot, w, lo);
      slot = q_next(slot);
    }
    __builtin_amdgcn_sched_barrier(0);
    // epilogue: h1 = ReLU(acc + b1) to HBM (columns 400 .. 415 zero), fm_y
    const int m = row0 + w * 16 + r16;
    int g4 = 4 * g;
    asm volatile("" : "+v"(g4));
    if (m < p.M) {
      float* hrow = p.H + (int64_t)m * kQN;
      uint32_t mb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int t = 0; t < kQNT; ++t) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 16 * t + g4);
        const f32x4 v = relu4(acc[t] + bb);
        *reinterpret_cast<f32x4*>(hrow + 16 * t + g4) = v;
        if constexpr (XS) {
          bits_set(mb, t, v);
          __builtin_amdgcn_sched_barrier(0);  // tile by tile (scheduled together, the bits spilled 177 SGPRs)
        }
      }
      *reinterpret_cast<f32x4*>(hrow + 16 * kQNT + g4) = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (XS)
        if (p.S) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<u32x4*>(p.S + ((int64_t)p.M + m) * 16 + g4) = u32x4{mb[0], mb[1], mb[2], mb[3]};
        }
    }
    {
#pragma clang fp contract(off)
      float a = 0.f;
      float d[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) d[t] = fs[t] * fs[t] - fq[t];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
#pragma unroll
        for (int t = 0; t < 4; ++t) a += __shfl(d[t], gg * 16 + r16);
      if (g == 0 && m < p.M && p.fm_y) p.fm_y[m] = p.fm_sums ? y1 + 0.5f * (a / 16.0f) : y1;
    }
    if constexpr (XS)
      if (p.S && m < p.M) *reinterpret_cast<f32x4*>(p.S + (int64_t)m * 16 + g4) = fs;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing DMAs land before the LDS is released
}

}  // namespace

bool tower_head_s3_usable(const DenseLayer& L1, int M, int F, int k, bool ids) {
  if (M <= 0 || !ids || k != 16 || F < 1 || F > kHMaxF || !L1.W3 || L1.W16 || !f32_split_enabled()) return false;
  if (!(L1.K == 16 * F && L1.N == 400 && L1.Npad == kQN && L1.N1 < 0 && L1.bias_mode == 1 && L1.K1 < 0)) return false;
  // knob "s3_head": 0 off, 2 always, 1 (default) when the (half) row blocks fill every CU at least once
  // (default 1 since measured: DeepFM B = 65,536 186.0 -> 188.2 M examples/s, layer 1 0.182 -> 0.173 ms,
  // profiles/r04/ab_round4_first.txt)
  const int knob = tuning_get("s3_head", 1);
  if (knob == 0) return false;
  if (knob == 2) return true;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  // (half) row blocks that fill every CU, or -- with half blocks -- any batch above the whole-tower kernel's
  // one round (k_small_s3.hip: M <= 16 ncu): half blocks on part of the chip still beat three engine launches
  return q_fills(M, ncu) || (tuning_get("half_blocks", 1) != 0 && M > 16 * ncu);
}

int launch_tower_head_s3(hipStream_t s, const DenseLayer& L1, int M, int F, const int32_t* ids, const float* table,
                         int ld, const float* wtab, int wld, float* H, int ldc, float* fm_y, int fm_sums, float* X,
                         int ldx, float* S) {
  if (!tower_head_s3_usable(L1, M, F, 16, ids != nullptr) && tuning_get("s3_head", 1) != 2) {
    set_error("fp32 tower head: needs a k = 16 gather (F <= 40, ids) into a 400-wide split-GEMM layer");
    return RMX_E_INVALID;
  }
  if (M <= 0) return RMX_OK;
  const int l = ld > 0 ? ld : 16, wl = wld > 0 ? wld : 1;
  if ((l & (l - 1)) || l < 16 || (wl & (wl - 1)) || ldc != kQN || !H) {
    set_error("fp32 tower head: table / weight strides must be powers of two, h1 [M][416]");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  if (X && ldx < 16 * F) {
    set_error("fp32 tower head: x needs ldx >= 16 F");
    return RMX_E_INVALID;
  }
  const void* fn = X ? (const void*)tower_head_s3_kernel<true> : (const void*)tower_head_s3_kernel<false>;
  RMX_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHLds));
  HeadS3Args p{};
  p.M = M;
  int grid = 0;
  p.rows = q_rows(M, ncu, grid);
  p.F = F;
  p.KS = (F + 1) / 2;
  p.ids = ids;
  p.table = table;
  p.gsh = __builtin_ctz((unsigned)l);
  p.wtab = wtab;
  p.wsh = __builtin_ctz((unsigned)wl);
  p.W = L1.W3;
  p.b = L1.b;
  p.H = H;
  p.fm_y = fm_y;
  p.fm_sums = fm_sums;
  p.X = X;
  p.ldx = ldx;
  p.S = S;
  if (X)
    hipLaunchKernelGGL(tower_head_s3_kernel<true>, dim3(grid), dim3(kQThreads), kHLds, s, p);
  else
    hipLaunchKernelGGL(tower_head_s3_kernel<false>, dim3(grid), dim3(kQThreads), kHLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
