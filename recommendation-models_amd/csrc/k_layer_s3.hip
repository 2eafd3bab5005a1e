// k_layer_s3.hip -- one 400 x 400 fp32 tower layer as a persistent row-owner kernel on the split GEMM (gfx950),
// for the training step (DeepFM training, BASELINE.json configs[1] at B = 65,536).
//
// Two uses of the same GEMM shape, C[M][416] from A[M][lda] (K = 400) and a 400-wide weight's split planes:
//   forward (EPI 0): h_l = ReLU(h_{l-1} W_l^T + b_l)            model/encoder/HigherOrderEncoder.scala:34-59,
//                    W = DenseLayer::W3; h_l is stored for the backward (the ReLU masks, the next dW)
//   dX (EPI 1):      dPre_{l-1} = (dPre_l W_l) * (h_{l-1} > 0)  the Linear + ReLU backward of
//                    deepfm/DeepFM.scala:83-124 (BigDL Linear.updateGradInput, ReLU.updateGradInput),
//                    W = DenseLayer::WT3 (W_l^T packed the same way)
// The ReLU mask travels as bits: the forward (and the training head, k_head_s3.hip) also stores
// hm[m][4 g + i] = the bits (h[m][16 t + 4 g + q] > 0) at position 4 t + q of the 128-bit word group of lane
// group g -- one 16-B store per lane, and one 16-B load per lane in the dX epilogue instead of 25 (read in
// five dependent groups next to the 100 accumulators, they cost the dX ~10 us per row block).
// The engine ran these at ~0.41-0.48 of the split peak (0.103 ms forward, 0.124 ms dX at B = 65,536); the
// row-owner tail (k_tail_s3.hip) runs its layers at ~0.6.  This is its layer-2 section on its own: a wave
// owns 16 rows and all 416 columns (operands swapped, D = W a^T), A streams from HBM by LDS-DMA into two
// per-wave step slots one unit ahead, the weights through the 3-slot unit ring (k_rowown.hpp), one barrier
// per unit, 26 units per 128-row block.  The epilogue stores the block's rows (EPI 1 loads the mask rows
// first); rows past M store to a sink and load a zero row, so every unit's vector-memory count is static.
// Products and K order are the tail's layer 2 (the engine's smallest-terms-first split order).
#include "k_rowown.hpp"

namespace rmx {
namespace {
using namespace rowown;

constexpr int kLKS = 13;                    // 32-wide K steps (K = 400, Kpad 416)
constexpr int kLUnits = 2 * kLKS;           // units per row block
constexpr int kLH = kQW * 2 * 2048;         // A: two 2-KiB step slots per wave
constexpr size_t kLLds = (size_t)kQSlots * kQUnit + kLH + sizeof(float) * kQN;
static_assert(kLLds <= 160 * 1024, "LDS budget");

__device__ __attribute__((aligned(16))) float g_lzero_row[kQN];   // A / mask rows past M
__device__ __attribute__((aligned(16))) float g_lsink[64 * 4];     // stores of rows past M

struct LayerS3Args {
  int M;
  QRows rows;
  const float* A;     // [M][lda] fp32, columns 0 .. 399 read (400 .. 415 zero-padded in the fragment)
  int lda;
  const bf16_t* W;    // [13][3][416][32] split planes
  const float* b;     // [416] (EPI 0)
  uint32_t* hm_out;         // EPI 0: [M][16] the ReLU mask bits of C (nullable: a sink)
  const uint32_t* hm_in;    // EPI 1: [M][16] the mask bits of the layer below: zero the outputs without one
  float* C;           // [M][ldc] out, columns 400 .. 415 zero
  int ldc;
};

__device__ __forceinline__ const bf16_t* l_unit_src(const LayerS3Args& p, int u) {
  const int c = u >> 1, half = u & 1;
  return p.W + (int64_t)(c * 3 * kQN + half * kQUT * 16) * 32;
}

// A of K step c of the row block at row0 into this wave's slot ds (k_tail_s3.hip q_h1_dma)
__device__ __forceinline__ void l_a_dma(const LayerS3Args& p, const float* zrow, char* alds, int row0, int nw, int c,
                                        int ds, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int r = 8 * i + (lane >> 3), j = (lane & 7) ^ ((lane >> 3) & 7);
    asm volatile("" : "+v"(r), "+v"(j));
    const int m = row0 + w * 16 + r;
    const uint32_t ok = (w < nw && m < p.M) ? 1u : 0u;
    const uintptr_t base = (uintptr_t)zrow + (uintptr_t)ok * ((uintptr_t)p.A - (uintptr_t)zrow);
    const float* row = reinterpret_cast<const float*>(base) + (uint32_t)(m * (int)ok) * (uint32_t)p.lda;
    lds_dma<16>(row + 32 * c + 4 * j, alds + ds * 2048 + i * 1024);
  }
}

__device__ __forceinline__ void l_a_read(const char* alds, int c, int lane, f32x4& a0, f32x4& a1) {
  const int r = lane & 15, g = lane >> 4;
  int o0 = r * 128 + ((g ^ (r & 7)) << 4), o1 = r * 128 + (((g + 4) ^ (r & 7)) << 4);
  asm volatile("" : "+v"(o0), "+v"(o1));
  a0 = *reinterpret_cast<const f32x4*>(alds + (c & 1) * 2048 + o0);
  a1 = *reinterpret_cast<const f32x4*>(alds + (c & 1) * 2048 + o1);
  if (c == kLKS - 1) a1 = f32x4{0.f, 0.f, 0.f, 0.f};
}

// vector-memory instructions of the epilogue, counted by the next block's first waits: EPI 0 26 row stores
// + the mask bits, EPI 1 the mask bits' load + 26 row stores
template <int EPI>
constexpr int kLEpi = kQNT + 2;


template <int EPI>
__global__ __launch_bounds__(kQThreads, 1) void layer_s3_kernel(LayerS3Args p) {
  extern __shared__ __attribute__((aligned(16))) char lsmem[];
  char* lds = lsmem;
  float* bl = reinterpret_cast<float*>(lsmem + kQSlots * kQUnit + kLH);
  const float* zrow = g_lzero_row;
  asm volatile("" : "+s"(zrow));
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int nit = p.rows.nit(blockIdx.x);

  if (EPI == 0)
    for (int i = tid; i < kQN; i += kQThreads) bl[i] = p.b ? p.b[i] : 0.f;
  int lo = (lane >> 2) * 32 + swz_slot(lane >> 2, lane & 3) * 8;
  asm volatile("" : "+v"(lo));
  const int fb = q_fbase(lane);
  char* alds = lsmem + kQSlots * kQUnit + w * 4096;
  {
    int row0, nw;
    p.rows.desc(blockIdx.x, 0, row0, nw);
    l_a_dma(p, zrow, alds, row0, nw, 0, 0, w, lane);
  }
  if (nit > 0) {
#pragma unroll
    for (int q = 0; q < kQQ; ++q) q_dma(l_unit_src(p, 0), lds, 0, w, q, lo);
#pragma unroll
    for (int q = 0; q < kQQ; ++q) q_dma(l_unit_src(p, 1), lds, 1, w, q, lo);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int slot = 0;
  for (int it = 0; it < nit; ++it) {
    int row0, nw, row0n, nwn;
    p.rows.desc(blockIdx.x, it, row0, nw);
    p.rows.desc(blockIdx.x, it + 1, row0n, nwn);
    if (w >= nw) {
      // a half block's waves 4 .. 7: the same units, barriers and DMAs, no MFMAs and no epilogue
#pragma unroll 1
      for (int c = 0; c < kLKS; ++c) {
        q_enter<5>();
        if (c + 1 < kLKS)
          l_a_dma(p, zrow, alds, row0, nw, c + 1, (c + 1) & 1, w, lane);
        else
          l_a_dma(p, zrow, alds, row0n, nwn, 0, 0, w, lane);
        __builtin_amdgcn_sched_barrier(0);
        int dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(l_unit_src(p, (2 * c + 2) % kLUnits), lds, dslot, w, lo);
        slot = q_next(slot);
        q_enter<7>();
        dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(l_unit_src(p, (2 * c + 3) % kLUnits), lds, dslot, w, lo);
        slot = q_next(slot);
      }
      continue;
    }
    f32x4 acc[kQNT];
#pragma unroll
    for (int t = 0; t < kQNT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c = 0; c < kLKS; ++c) {
      // previous unit: (c - 1, half 1): 5 DMAs; at c = 0 the previous block's last unit + its epilogue
      if (c == 0)
        q_enter<5 + kLEpi<EPI>>();
      else
        q_enter<5>();
      bf16x8 ah, am, al;
      {
        f32x4 a0, a1;
        l_a_read(alds, c, lane, a0, a1);
        split3(a0, a1, ah, am, al);
      }
      // the next step's A, or the next row block's step 0 into the slot just read (step 12 is slot 0)
      if (c + 1 < kLKS)
        l_a_dma(p, zrow, alds, row0, nw, c + 1, (c + 1) & 1, w, lane);
      else
        l_a_dma(p, zrow, alds, row0n, nwn, 0, 0, w, lane);
      __builtin_amdgcn_sched_barrier(0);
      const int u = 2 * c;
      int dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQUT, 0>(lds + slot * kQUnit, fb, ah, am, al, acc, l_unit_src(p, (u + 2) % kLUnits), lds, dslot, w, lo);
      slot = q_next(slot);
      q_enter<7>();  // previous unit: 2 A loads + 5 DMAs
      dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQNT - kQUT, kQUT>(lds + slot * kQUnit, fb, ah, am, al, acc, l_unit_src(p, (u + 3) % kLUnits), lds, dslot,
                                w, lo);
      slot = q_next(slot);
    }
    __builtin_amdgcn_sched_barrier(0);
    // epilogue: every lane issues the same loads / stores (rows past M: the zero row / the sink)
    // (global address space explicitly: the zero row's pointer went through asm and would make these flat)
    typedef __attribute__((address_space(1))) f32x4 gf32x4;
    const int m = row0 + w * 16 + r16;
    const bool ok = m < p.M;
    int g4 = 4 * g;
    asm volatile("" : "+v"(g4));
    gf32x4* crow = reinterpret_cast<gf32x4*>(ok ? reinterpret_cast<uintptr_t>(p.C + (int64_t)m * p.ldc + g4)
                                                : reinterpret_cast<uintptr_t>(g_lsink + lane * 4));
    const int cstep = ok ? 4 : 0;  // (f32x4 units)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) u32x4 guint4;
    if constexpr (EPI == 0) {
      uint32_t mb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int t = 0; t < kQNT; ++t) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 16 * t + g4);
        const f32x4 v = relu4(acc[t] + bb);
        bits_set(mb, t, v);
        crow[cstep * t] = v;
      }
      guint4* hb = reinterpret_cast<guint4*>(ok && p.hm_out ? reinterpret_cast<uintptr_t>(p.hm_out + (int64_t)m * 16 + g4)
                                                            : reinterpret_cast<uintptr_t>(g_lsink + 64 * 4 - 4));
      *hb = u32x4{mb[0], mb[1], mb[2], mb[3]};
    } else {
      const guint4* hb = reinterpret_cast<const guint4*>(ok ? reinterpret_cast<uintptr_t>(p.hm_in + (int64_t)m * 16 + g4)
                                                            : reinterpret_cast<uintptr_t>(zrow));
      const u32x4 mv = *hb;
      const uint32_t mb[4] = {mv[0], mv[1], mv[2], mv[3]};
#pragma unroll
      for (int t = 0; t < kQNT; ++t) {
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 4 * t + q;
          v[q] = ((mb[i >> 5] >> (i & 31)) & 1u) ? acc[t][q] : 0.f;
        }
        crow[cstep * t] = v;
      }
    }
    crow[cstep * kQNT] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool layer_s3_usable(const DenseLayer& L, bool dx, int M, int lda, int ldc) {
  // knob "train_layer_s3": 1 (default) forward and dX, 2 forward only, 0 off
  const int knob = tuning_get("train_layer_s3", 1);
  if (knob == 0 || (dx && knob == 2)) return false;
  const bf16_t* W = dx ? L.WT3 : L.W3;
  if (M <= 0 || !W || L.W16 || !f32_split_enabled()) return false;
  if (!(L.K == 400 && L.N == 400 && L.Npad == kQN && L.N1 < 0 && L.bias_mode == 1 && lda >= kQN && lda % 4 == 0 &&
        ldc >= kQN && ldc % 4 == 0))
    return false;
  if (dx ? (L.NTpad != kQN || (L.KTpad / 16 + 1) / 2 != kLKS) : (L.Kpad + 31) / 32 != kLKS) return false;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  return q_fills(M, ncu) && (int64_t)M * lda < ((int64_t)1 << 31);
}

int launch_layer_s3(hipStream_t s, const DenseLayer& L, bool dx, int M, const float* A, int lda, float* C, int ldc,
                    uint32_t* hm_out, const uint32_t* hm_in) {
  if (!layer_s3_usable(L, dx, M, lda, ldc)) {
    set_error("fp32 row-owner layer: needs a 400 x 400 split-GEMM layer, [M][>= 416] operands and a full round of row blocks");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  LayerS3Args p{};
  p.M = M;
  int grid = 0;
  p.rows = q_rows(M, ncu, grid);
  p.A = A;
  p.lda = lda;
  p.W = dx ? L.WT3 : L.W3;
  p.b = L.b;
  p.hm_out = hm_out;
  p.hm_in = hm_in;
  p.C = C;
  p.ldc = ldc;
  if (dx && hm_in) {
    RMX_HIP(hipFuncSetAttribute((const void*)layer_s3_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLLds));
    hipLaunchKernelGGL(layer_s3_kernel<1>, dim3(grid), dim3(kQThreads), kLLds, s, p);
  } else if (!dx) {
    RMX_HIP(hipFuncSetAttribute((const void*)layer_s3_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLLds));
    hipLaunchKernelGGL(layer_s3_kernel<0>, dim3(grid), dim3(kQThreads), kLLds, s, p);
  } else {
    set_error("fp32 row-owner layer: dX needs the ReLU mask bits of the layer below");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
