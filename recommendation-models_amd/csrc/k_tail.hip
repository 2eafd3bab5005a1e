// k_tail.hip -- the bf16 tower tail in one persistent kernel (BASELINE.json configs[4]: DCN / PNN
// bf16, gfx950).
//
// The last hidden Linear + ReLU and the output Linear + head of a bf16 tower
// (model/encoder/HigherOrderEncoder.scala:34-59: Linear(400 -> 400) + ReLU, then the last
// Linear(400 -> 400) + ReLU whose output feeds Linear(400 -> 1); the heads of DCN.scala /
// PNN.scala: CAddTable + Sigmoid) as ONE launch over row blocks of 64 samples:
//   h2 = bf16(ReLU(h1 W2^T + b2))        kept in LDS, never written to HBM
//   y  = sum_n ReLU(h2 W3^T + b3)[n] wo[n] (+ bo) ; p = sigmoid(pre + (pre2 + y) + beta)
// Why: run as two launches, each layer reads 52 MB and the first writes 52 MB at B = 65,536, with
// one stage of 30 KiB in flight per block (26 KiB of it the weights from L2), so both layers sat
// at ~2.9 TB/s and 0.2 of the bf16 peak, bound by memory latency rather than by HBM or MFMA.
// Here the only HBM traffic is h1 (read once) and p.
//
// Block = 16 waves on one CU (persistent: grid = min(row blocks, CUs)):
//   - 4 loader waves (one per SIMD) DMA the NEXT row block's h1 tile (64 rows x 416 bf16 = 52 KiB,
//     global_load_lds) into the idle half of a double-buffered LDS image while the 12 compute waves
//     run the current one, so the tile's HBM latency hides behind two layers of MFMAs (a loader's
//     vmcnt wait stalls only the loader: every wave has its own counter);
//   - compute wave w owns column tiles w, w + 12, w + 24 (< 26) of both layers for all 64 rows:
//     waves 0-1 three tiles, 2-11 two, i.e. 7 / 7 / 6 / 6 tiles per SIMD (waves w and w + 4 share
//     a SIMD);
//   - the weights (W2, W3: [13 steps][416][32] bf16, 338 KiB each, L2-resident) go straight from
//     global memory into registers, two K steps ahead: each fragment is 1 KiB contiguous per wave
//     and exactly one wave of the block reads it, so staging it through LDS would buy no reuse;
//   - the MFMA runs with the operands swapped (D = W h^T: v_mfma_f32_16x16x32_bf16 with the weight
//     fragment as A), so a lane ends up holding 4 consecutive outputs n of one sample, which is
//     what the epilogue needs: h2 goes back into the tile's own LDS image as one 8-B bf16x4 write
//     per (tile, row tile), and the output dot sums along the lane first.
// Per K step a compute wave reads 4 A fragments (4 KiB) from LDS and issues 4 x NTW MFMAs; per SIMD
// that is 28 MFMAs x 16 cycles against 16 KiB of LDS reads (128 cycles at 128 B/clk): MFMA-bound.
// The sums are the unfused kernels' up to the order of the final logit reduction: h2 is the same
// bf16 (RNE) of the same fp32 accumulations (K steps in order), so parity is held to the same bar
// against the oracle's bf16 emulation (tests/test_bf16.py).
#include "k_gemm.hpp"

namespace rmx {
namespace {

constexpr int kTBM = 64;                   // rows per row block
constexpr int kTNT = 26;                   // 16-column tiles: Npad = 416 (N <= 416)
constexpr int kTKS = 13;                   // 32-wide K steps: Kpad = 416
constexpr int kTN = kTNT * 16;
constexpr int kTCW = 12;                   // compute waves
constexpr int kTLW = 4;                    // loader waves
constexpr int kTThreads = (kTCW + kTLW) * 64;
constexpr int kTImg = kTKS * kTBM * 64;    // bytes of one h tile image [step][row][64 B] (53,248)
constexpr int kTIns = kTImg / 1024;        // 1-KiB DMA instructions per image (52)
// weight fragments are loaded PF K steps ahead: 2 for the two-tile waves, 1 for the three-tile ones
// (2 spills there at the 128-VGPR budget of 4 waves per SIMD)
template <int NTW>
constexpr int kTPF = NTW >= 3 ? 1 : 2;
constexpr size_t kTLds = 2 * kTImg + sizeof(float) * kTCW * kTBM;

static_assert(kTIns % kTLW == 0, "every loader issues the same DMAs");

struct TailArgs {
  int M, nblk;
  const bf16_t* H;  // layer input [M][lda] bf16; columns >= K2 read as zero
  int lda, K2;
  const bf16_t* W2;  // [13][416][32]
  const float* b2;   // [416]
  const bf16_t* W3;
  const float* b3;
  OutArgs oa;        // wo [416], bo, pre, pre2, rowsum, beta, out
};

__device__ __forceinline__ void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// weight fragment of K step c, the wave's column tile j: Wl = this lane's element of the wave's
// first tile (W + ((w * 16 + r16) * 32 + g * 8)); tile j is 12 tiles further: 1 KiB per wave
__device__ __forceinline__ f32x4 ldw(const bf16_t* Wl, int c, int j) {
  return *reinterpret_cast<const f32x4*>(Wl + (c * kTN + j * kTCW * 16) * 32);
}
// the lane's base of ldw, opaque to the optimiser so that the 13 x NTW fragment addresses are formed
// step by step instead of being hoisted out of the row-block loop (which spilled)
__device__ __forceinline__ const bf16_t* wlane(const bf16_t* W, int w, int lane) {
  const bf16_t* Wl = W + ((w * 16 + (lane & 15)) * 32 + (lane >> 4) * 8);
  asm volatile("" : "+v"(Wl));
  return Wl;
}
// h fragment of K step c for tile row `row`, k slot g, from a swizzled image
__device__ __forceinline__ f32x4 ldh(const char* img, int c, int row, int g) {
  return *reinterpret_cast<const f32x4*>(img + ((c * kTBM + row) * 4 + swz_slot(row, g)) * 16);
}

// one layer's K loop: acc[i][j] (tile row i, column tile j) += W_j h_i^T over the 13 steps; wb holds
// the prologue's fragments of steps 0 .. kTPF - 1 on entry
template <int NTW>
__device__ __forceinline__ void tail_layer(const bf16_t* Wl, const char* img, int lane,
                                           f32x4 (&acc)[4][NTW], f32x4 (&wb)[kTPF<NTW> + 1][NTW]) {
  const int g = lane >> 4, r16 = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kTKS; ++c) {
    if (c + kTPF<NTW> < kTKS)
#pragma unroll
      for (int j = 0; j < NTW; ++j) wb[(c + kTPF<NTW>) % (kTPF<NTW> + 1)][j] = ldw(Wl, c + kTPF<NTW>, j);
    f32x4 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ldh(img, c, 16 * i + r16, g);
    __builtin_amdgcn_sched_barrier(0);  // one step's loads at a time (hoisting them all spills)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wb[c % (kTPF<NTW> + 1)][j]),
                                                            __builtin_bit_cast(bf16x8, a[i]), acc[i][j], 0, 0, 0);
  }
}

template <int NTW>
__device__ __forceinline__ void tail_prologue(const bf16_t* Wl, f32x4 (&wb)[kTPF<NTW> + 1][NTW]) {
#pragma unroll
  for (int c = 0; c < kTPF<NTW>; ++c)
#pragma unroll
    for (int j = 0; j < NTW; ++j) wb[c][j] = ldw(Wl, c, j);
}

template <int NTW>
__device__ void tail_compute(const TailArgs& p, char* smem, int w, int lane, int nit) {
  const int g = lane >> 4, r16 = lane & 15;
  float* red = reinterpret_cast<float*>(smem + 2 * kTImg);  // [kTCW][kTBM] partial logits
  f32x4 acc[4][NTW];
  f32x4 wb[kTPF<NTW> + 1][NTW];
  tail_prologue<NTW>(wlane(p.W2, w, lane), wb);
  for (int it = 0; it < nit; ++it) {
    const int rb = blockIdx.x + it * gridDim.x;
    char* img = smem + (it & 1) * kTImg;
    __builtin_amdgcn_s_barrier();  // B0: the loaders' DMAs of this tile have landed
    asm volatile("" ::: "memory");
    tail_layer<NTW>(wlane(p.W2, w, lane), img, lane, acc, wb);
    tail_prologue<NTW>(wlane(p.W3, w, lane), wb);  // in flight across the epilogue
    bar_lds();                              // B1: every wave has read the tile
    // h2 = bf16(ReLU(acc + b2)) into the same image: lane holds n = 16 t + 4 g .. + 3 of row 16 i + r16
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n0 = 16 * (w + kTCW * j) + 4 * g;
      const f32x4 bb = p.b2 ? *reinterpret_cast<const f32x4*>(p.b2 + n0) : f32x4{0.f, 0.f, 0.f, 0.f};
      const int c = n0 >> 5, slot = (n0 & 31) >> 3, half = (n0 >> 2) & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + r16;
        f32x4 v = acc[i][j] + bb;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
        *reinterpret_cast<bf16x4*>(img + ((c * kTBM + row) * 4 + swz_slot(row, slot)) * 16 + half * 8) =
            __builtin_convertvector(v, bf16x4);
      }
    }
    bar_lds();  // B2: h2 complete
    tail_layer<NTW>(wlane(p.W3, w, lane), img, lane, acc, wb);
    if (it + 1 < nit) tail_prologue<NTW>(wlane(p.W2, w, lane), wb);
    // output dot: part[i] = sum over this lane's n of ReLU(acc + b3)[n] * wo[n], then over the 4 lane groups
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n0 = 16 * (w + kTCW * j) + 4 * g;
      const f32x4 bb = p.b3 ? *reinterpret_cast<const f32x4*>(p.b3 + n0) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 wv = *reinterpret_cast<const f32x4*>(p.oa.wo + n0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bb[r];
          v = v > 0.f ? v : 0.f;
          part[i] += v * wv[r];
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      part[i] += __shfl_xor(part[i], 16);
      part[i] += __shfl_xor(part[i], 32);
      if (g == 0) red[w * kTBM + 16 * i + r16] = part[i];
    }
    bar_lds();  // B3: partial logits complete
    if (w == 0) {
      const int m = rb * kTBM + lane;
      if (m < p.M) {
        const OutArgs& oa = p.oa;
        float y = red[lane];
#pragma unroll
        for (int q = 1; q < kTCW; ++q) y += red[q * kTBM + lane];
        if (oa.has_bo) y = y + oa.bo;
        if (oa.rowsum) {
          float rs = 0.f;
          for (int jj = 0; jj < oa.rowsum_k; ++jj) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + jj];
          y = rs + y;
        }
        if (oa.pre2) y = oa.pre2[m] + y;
        float t = oa.pre ? oa.pre[m] + y : y;
        t = t + oa.beta;
        oa.out[m] = 1.0f / (1.0f + expf(-t));
      }
    }
  }
}

// loader wave lw: its share (13 of the 52 1-KiB instructions) of row block rb's h tile into image
// `img`; lane L of instruction ins fills image row R = 16 ins + L / 4 (R = step * 64 + row) at
// physical slot L & 3, i.e. loads logical slot swz_slot(row, L & 3) (the swizzle is an involution)
__device__ void tail_issue(const TailArgs& p, char* img, int rb, int lw, int lane, const float* zero16) {
  const int m0 = rb * kTBM;
#pragma unroll
  for (int q = 0; q < kTIns / kTLW; ++q) {
    const int ins = lw + kTLW * q;
    const int R = ins * 16 + (lane >> 2);
    const int c = R / kTBM, row = R - c * kTBM;
    const int m = m0 + row, kk = c * 32 + swz_slot(row, lane & 3) * 8;
    const void* src = (m < p.M && kk < p.K2) ? (const void*)(p.H + (int64_t)m * p.lda + kk) : (const void*)zero16;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(img + ins * 1024), 16, 0, 0);
  }
}

__global__ __launch_bounds__(kTThreads, 1) void tower_tail_bf16_kernel(TailArgs p) {
  extern __shared__ __attribute__((aligned(16))) char tsmem[];
  const float* zero16 = g_rmx_zero16;
  asm volatile("" : "+s"(zero16));
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nit = blockIdx.x < p.nblk ? (p.nblk - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (w < 2) {
    tail_compute<3>(p, tsmem, w, lane, nit);
  } else if (w < kTCW) {
    tail_compute<2>(p, tsmem, w, lane, nit);
  } else {
    // loaders: tile it + 1 streams in while the compute waves run tile it; every wave passes the
    // same four barriers per tile (B0 .. B3)
    const int lw = w - kTCW;
    if (nit > 0) tail_issue(p, tsmem, blockIdx.x, lw, lane, zero16);
    for (int it = 0; it < nit; ++it) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // B0
      if (it + 1 < nit) tail_issue(p, tsmem + ((it + 1) & 1) * kTImg, blockIdx.x + (it + 1) * gridDim.x, lw, lane, zero16);
      __builtin_amdgcn_s_barrier();  // B1
      __builtin_amdgcn_s_barrier();  // B2
      __builtin_amdgcn_s_barrier();  // B3
    }
  }
}

}  // namespace

bool tower_tail_usable(const DenseLayer& L2, const DenseLayer& L3, int M, int lda) {
  return tuning_get("bf16_tail", 1) != 0 && M > 0 && L2.W16 && L3.W16 && L2.Npad == kTN && L3.Npad == kTN &&
         L2.Kpad == kTKS * 32 && L3.Kpad == kTKS * 32 && L3.K <= L2.Npad && lda >= L2.K && lda % 8 == 0 &&
         L2.N1 < 0 && L3.N1 < 0;
}

int launch_tower_tail_bf16(hipStream_t s, const DenseLayer& L2, const DenseLayer& L3, int M, const bf16_t* H, int lda,
                           const OutArgs& oa) {
  if (!tower_tail_usable(L2, L3, M, lda) || !oa.wo || !oa.out) {
    set_error("tower tail: needs two bf16 layers of Npad = Kpad = 416 and an output head");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  RMX_HIP(hipFuncSetAttribute((const void*)tower_tail_bf16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kTLds));
  TailArgs p{};
  p.M = M;
  p.nblk = (M + kTBM - 1) / kTBM;
  p.H = H;
  p.lda = lda;
  p.K2 = L2.K;
  p.W2 = L2.W16;
  p.b2 = L2.b;
  p.W3 = L3.W16;
  p.b3 = L3.b;
  p.oa = oa;
  const int grid = std::min(p.nblk, std::max(ncu, 1));
  hipLaunchKernelGGL(tower_tail_bf16_kernel, dim3(grid), dim3(kTThreads), kTLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
