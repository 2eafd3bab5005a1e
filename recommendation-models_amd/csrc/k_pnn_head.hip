// k_pnn_head.hip -- PNN's tower layer 1 with the inner products generated on chip (gfx950), BASELINE.json
// configs[4] (bf16).
//
// The reference builds PNN's layer-1 input as [x || ip]: x = the F gathered k = 16 rows and ip = the
// F (F - 1) / 2 pair dot products e_i . e_j, i < j (pnn/ProductEncoder.scala:72-120 over bnn/Gather.scala:35-42
// and bnn/DotProduct2.scala:16-26), then Linear(D + P -> N1) + ReLU (HigherOrderEncoder.scala:34-59).  The
// unfused path materialises that 2,816-B row per sample in HBM (product16_kernel) and the column-sliced
// GEMM reads it back.  Here the row never leaves the CU:
//   * a block of 4 waves (one per SIMD) owns 64 samples; a wave owns 16 samples and all 416 columns, MFMA
//     operands swapped (D = W x^T, v_mfma_f32_16x16x32_bf16), as in k_head_bf16.hip;
//   * the wave's 16 x F rows (bf16) stay resident in its LDS image [40 fields][2 halves][16 samples][16 B]
//     (20 KiB); the x steps (K = 32 per unit: fields 2c, 2c + 1) read their B fragment from it, and the ip
//     steps' B fragments are computed from it on the VALU one unit ahead (v_dot2c_f32_bf16, fp32, rounded to
//     bf16 once -- the storage point of the bf16 oracle and of product16_kernel);
//   * the ip K order is "quads": 4 pairs (i, j0 .. j0 + 3) of one row i, so a lane computes its 8 B values
//     from 2 rows i and 8 rows j.  The weights are packed in that order at set_mats (PnnHead::W; zero for the
//     padded j >= F and pad quads): 200 quads = 25 ip units at F = 39 against 24 for the dense order;
//   * the next row block's rows are gathered into the fields this block has finished with: a field is free
//     once the quads of its last row i are done, and the next block needs its pairs in x order, so every
//     pair gets >= 15 units of lead at F = 39 (the per-unit schedule PnnHead::sched, built on the host);
//   * weights stream through a 3-slot LDS ring (26 KiB per unit, 7 DMAs per wave), one barrier per unit.
// LDS: 3 x 26,624 + 4 x (20,480 + 512) = 163,840 B.
#include "k_rowown.hpp"

#include <vector>

namespace rmx {
namespace {
using namespace rowown;

constexpr int kPW = 4;                          // waves per block (one per SIMD)
constexpr int kPThreads = kPW * 64;
constexpr int kPBM = kPW * 16;                  // samples per row block
constexpr int kPNT = 26;                        // column tiles (416)
constexpr int kPUnit = kPNT * 1024;             // one K step of the packed weights
constexpr int kPIns = kPUnit / 1024;            // 26 DMA instructions per unit
constexpr int kPQ = (kPIns + kPW - 1) / kPW;    // 7 per wave (waves 2, 3 repeat instruction 25)
constexpr int kPSlots = 3;
constexpr int kPMaxF = 40;
constexpr int kPRows = kPMaxF * 512;            // per wave: [40 fields][2 halves][16 samples][16 B]
constexpr int kPIds = 4 * 128;                  // per wave: 4 id slots x [2 fields][16 samples]
constexpr int kPWave = kPRows + kPIds;
constexpr size_t kPLds = (size_t)kPSlots * kPUnit + (size_t)kPW * kPWave;
static_assert(kPLds <= 160 * 1024, "LDS budget");
static_assert(kPQ == 7, "the static vmcnt count below assumes 7 weight DMAs per wave per unit");
constexpr int kNone = 127;

struct PnnArgs {
  int M, nblk, F, KSX, KS;
  const int32_t* ids;     // [M][F]
  const bf16_t* table;    // row of id at table + id * 16
  const bf16_t* W;        // [KS][416][32] (PnnHead::W)
  const float* b;         // [416]
  int N1;                 // columns stored ReLU'd; the rest zero
  bf16_t* H;              // [M][416]
  const int32_t* quads;   // [(KS - KSX) * 8]: i | j0 << 8
  const int32_t* sched;   // [KS]: row pair | id pair << 8 | id-of-next-block << 15 (pair kNone: none)
  const int32_t* pro;     // [KSX]: 2 = the prologue gathers pair c's rows, 1 = its ids, 0 = nothing
};

__device__ __forceinline__ void p_wdma(const bf16_t* src, char* lds, int slot, int w, int q) {
  int ins = w + q * kPW;
  ins = ins < kPIns ? ins : kPIns - 1;
  int lo = (threadIdx.x & 63) >> 2;  // row of the tile; physical slot lane & 3 holds logical swz_slot(row, .)
  lo = lo * 32 + swz_slot(lo, threadIdx.x & 3) * 8;
  asm volatile("" : "+v"(lo));
  lds_dma<16>(src + ins * 16 * 32 + lo, lds + slot * kPUnit + ins * 1024);
}

// ids of pair c (fields 2c, 2c + 1) of row block rb into id slot c & 3 (lanes 0 .. 31: field 2c + (L >> 4),
// sample L & 15)
__device__ __forceinline__ void p_id_dma(const PnnArgs& p, char* wl, int rb, int c, int w, int lane) {
  int f = lane >> 4, s = lane & 15;
  asm volatile("" : "+v"(f), "+v"(s));
  const int m = rb * kPBM + w * 16 + s, fld = 2 * c + f;
  const bool ok = rb < p.nblk && m < p.M && fld < p.F;
  const int32_t* src = ok ? p.ids + (int64_t)m * p.F + fld : g_rmx_neg1;
  if (lane < 32) lds_dma<4>(src, wl + kPRows + (c & 3) * 128);
}

// rows of pair c from the ids in slot c & 3: lane L = field 2c + (L >> 5), half (L >> 4) & 1, sample L & 15
// lands at image byte c * 1024 + 16 L
__device__ __forceinline__ void p_row_dma(const PnnArgs& p, char* wl, int c, int lane) {
  const int* ids = reinterpret_cast<const int*>(wl + kPRows + (c & 3) * 128);
  int f = lane >> 5, h = (lane >> 4) & 1, s = lane & 15;
  asm volatile("" : "+v"(f), "+v"(h), "+v"(s));
  const int id = ids[f * 16 + s];
  const void* src = id >= 0 ? (const void*)(p.table + ((int64_t)id << 4) + 8 * h) : (const void*)g_rmx_zero16;
  lds_dma<16>(src, wl + c * 1024);
}

// the prologue's rows of pair c of row block rb, ids read straight from HBM
__device__ __forceinline__ void p_row_direct(const PnnArgs& p, char* wl, int rb, int c, int w, int lane) {
  const int f = lane >> 5, h = (lane >> 4) & 1, s = lane & 15;
  const int m = rb * kPBM + w * 16 + s, fld = 2 * c + f;
  const int id = (rb < p.nblk && m < p.M && fld < p.F) ? p.ids[(int64_t)m * p.F + fld] : -1;
  const void* src = id >= 0 ? (const void*)(p.table + ((int64_t)id << 4) + 8 * h) : (const void*)g_rmx_zero16;
  lds_dma<16>(src, wl + c * 1024);
}

template <int N>
__device__ __forceinline__ void p_enter() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// e_i . e_j of one sample, 16 bf16 as 2 x 4 dwords each, pairwise in element order, fp32.  (The dwords are
// named explicitly: __builtin_bit_cast of a vector-element subscript v[q] read element 0 for every q here.)
__device__ __forceinline__ float p_dot(const u32x4 (&a)[2], const u32x4 (&b)[2]) {
  float d = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const unsigned int av[4] = {a[h].x, a[h].y, a[h].z, a[h].w}, bv[4] = {b[h].x, b[h].y, b[h].z, b[h].w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, av[q]), __builtin_bit_cast(bf16x2, bv[q]), d,
                                          false);
  }
  return d;
}

// uniform table reads through the scalar cache (a vector load here would make the compiler drain vmcnt --
// every DMA in flight -- before the value is used)
__device__ __forceinline__ int p_sld(const int32_t* base, int i) {
  const __attribute__((address_space(4))) int32_t* c = (const __attribute__((address_space(4))) int32_t*)base;
  return c[__builtin_amdgcn_readfirstlane(i)];
}

// One unit t of a row block.  The B fragment is x (pair t of the image) for t < KSX, else the ip fragment
// computed by the previous unit; when unit t + 1 is an ip unit its fragment is computed here on the side
// (quads from p.quads).  One loop runs every unit, the ip work under uniform per-tile branches: two loops
// over the two kinds, or the two kinds as two bodies under one branch, made the compiler copy the 104
// accumulators between VGPRs and AGPRs every unit.
__device__ __forceinline__ void p_unit(const PnnArgs& p, char* smem, char* wl, const char* rl, int t, int rb, int rbn,
                                       int& slot, int fb, int lane, int w, f32x4 (&acc)[kPNT], bf16x8& ipf) {
  p_enter<kPQ>();  // all but this wave's last 7 DMAs (the previous unit's weights) have landed
  const int sc = p_sld(p.sched, t);
  const bool xb = t < p.KSX, ipn = t + 1 >= p.KSX && t + 1 < p.KS;
  int xo = (xb ? t : 0) * 1024 + lane * 16;
  asm volatile("" : "+v"(xo));
  const bf16x8 xf = *reinterpret_cast<const bf16x8*>(wl + xo);
  const bf16x8 bfr = xb ? xf : ipf;
  const int rp = sc & 127, ipr = (sc >> 8) & 127;
  if (rp != kNone) p_row_dma(p, wl, rp, lane);
  if (ipr != kNone) p_id_dma(p, wl, (sc >> 15) & 1 ? rbn : rb, ipr, w, lane);
  // this unit's weight DMAs (unit t + 2) all here, ahead of the fragment reads: interleaved with them, each
  // LDS DMA made the compiler drain lgkmcnt -- the prefetched fragments -- before the next MFMA
  const int ds = slot == 0 ? 2 : slot - 1;  // (slot + 2) mod 3
  const int tn = t + 2 < p.KS ? t + 2 : t + 2 - p.KS;
  const bf16_t* src = p.W + (int64_t)tn * kQN * 32;
#pragma unroll
  for (int q = 0; q < kPQ; ++q) p_wdma(src, smem, ds, w, q);
  __builtin_amdgcn_sched_barrier(0);
  const char* ub = smem + slot * kPUnit;
  int fbu = fb;
  asm volatile("" : "+v"(fbu));
  // ip of unit t + 1: lane (r16, g) computes K positions 8 g .. 8 g + 7 = quads 2 g, 2 g + 1 of that step
  int qi[2] = {0, 0}, qj[2] = {0, 0};
  if (ipn) {
    const int q0 = (t + 1 - p.KSX) * 8, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int a0 = p_sld(p.quads, q0 + u), a1 = p_sld(p.quads, q0 + 2 + u);
      const int a2 = p_sld(p.quads, q0 + 4 + u), a3 = p_sld(p.quads, q0 + 6 + u);
      const int q = g == 0 ? a0 : (g == 1 ? a1 : (g == 2 ? a2 : a3));
      qi[u] = q & 255;
      qj[u] = q >> 8;
    }
  }
  u32x4 ri[2], rj[2][2];
  float ipv[8];
  auto rd_row = [&](int fld, u32x4 (&r)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) r[h] = *reinterpret_cast<const u32x4*>(rl + fld * 512 + h * 256);
  };
  auto jfld = [&](int e) {
    const int j = qj[e >> 2] + (e & 3);
    return j < p.F ? j : p.F - 1;  // padded positions: any finite value (their weights are zero)
  };
  constexpr int PF = 3;
  f32x4 bq[PF + 1];
#pragma unroll
  for (int tt = 0; tt < PF; ++tt) bq[tt] = *reinterpret_cast<const f32x4*>(ub + fbu + tt * 1024);
#pragma unroll
  for (int tt = 0; tt < kPNT; ++tt) {
    if (tt + PF < kPNT) bq[(tt + PF) % (PF + 1)] = *reinterpret_cast<const f32x4*>(ub + fbu + (tt + PF) * 1024);
    // pair e: rows read at tile 3 e, dot at tile 3 e + 2; row i of quad u at tiles 0 / 12 (quad 1's row
    // replaces quad 0's after pair 3's dot at tile 11)
    if (ipn) {
      if (tt == 0) rd_row(qi[0], ri);
      if (tt == 12) rd_row(qi[1], ri);
      if (tt % 3 == 0 && tt / 3 < 8) rd_row(jfld(tt / 3), rj[(tt / 3) & 1]);
      if (tt % 3 == 2 && tt / 3 < 8) ipv[tt / 3] = p_dot(ri, rj[(tt / 3) & 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bq[tt % (PF + 1)]), bfr, acc[tt], 0, 0,
                                                      0);
  }
  if (ipn) {
    typedef float f32x8 __attribute__((ext_vector_type(8)));
    f32x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ipv[e];
    ipf = __builtin_convertvector(v, bf16x8);
  }
  slot = slot == kPSlots - 1 ? 0 : slot + 1;
}

__global__ __launch_bounds__(kPThreads, 1) void pnn_head_kernel(PnnArgs p) {
  extern __shared__ __attribute__((aligned(16))) char psmem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  char* wl = psmem + kPSlots * kPUnit + w * kPWave;
  const char* rl = wl + r16 * 16;  // this lane's sample in the row image
  const int nit = (int)blockIdx.x < p.nblk ? (p.nblk - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int fb = q_fbase(lane);
  // PNN's layer-1 bias is one scalar broadcast over the N1 columns (CAdd(1): bias_mode 2)
  const float b0 = __int_as_float(p_sld(reinterpret_cast<const int32_t*>(p.b), 0));
  if (nit > 0) {
    for (int c = 0; c < p.KSX; ++c) {
      const int a = p_sld(p.pro, c);
      if (a == 2) p_row_direct(p, wl, blockIdx.x, c, w, lane);
      if (a == 1) p_id_dma(p, wl, blockIdx.x, c, w, lane);
    }
#pragma unroll
    for (int q = 0; q < kPQ; ++q) {
      p_wdma(p.W, psmem, 0, w, q);
      p_wdma(p.W + (int64_t)(1 % p.KS) * kQN * 32, psmem, 1, w, q);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int slot = 0;
  bf16x8 ipf = {};
  for (int it = 0; it < nit; ++it) {
    const int rb = blockIdx.x + it * gridDim.x, rbn = rb + gridDim.x;
    f32x4 acc[kPNT];
#pragma unroll
    for (int t = 0; t < kPNT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int t = 0; t < p.KS; ++t) p_unit(p, psmem, wl, rl, t, rb, rbn, slot, fb, lane, w, acc, ipf);
    __builtin_amdgcn_sched_barrier(0);
    const int m = rb * kPBM + w * 16 + r16;
    if (m < p.M) {
      bf16_t* hrow = p.H + (int64_t)m * kQN;
#pragma unroll
      for (int t = 0; t < kPNT; ++t) {
        int n0 = 16 * t + 4 * g;
        asm volatile("" : "+v"(n0));
        f32x4 v = acc[t];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = n0 + r < p.N1 && v[r] + b0 > 0.f ? v[r] + b0 : 0.f;
        *reinterpret_cast<bf16x4*>(hrow + n0) = __builtin_convertvector(v, bf16x4);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// W[n][kx] of PNN's layer 1 (Linear(x) + Linear(ip) side by side: LayerUtil offsets, k_encoder.hip layer_w)
__global__ void pnn_pack_kernel(const float* __restrict__ mats, DenseLayer L, const int* __restrict__ colmap, int KS,
                                bf16_t* __restrict__ Wp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)KS * 32 * kQN) return;
  const int kk = (int)(i & 31);
  const int64_t rest = i >> 5;
  const int n = (int)(rest % kQN), c = (int)(rest / kQN);
  const int kx = colmap[c * 32 + kk];
  float v = 0.f;
  if (kx >= 0 && n < L.N)
    v = kx < L.K1 ? mats[L.w_off + (int64_t)n * L.K1 + kx] : mats[L.w_off2 + (int64_t)n * (L.K - L.K1) + (kx - L.K1)];
  Wp[i] = (bf16_t)v;
}

// The quads, the packed K order and the per-unit DMA schedule for F (see the header); false when F does
// not fit the image or a pair would miss its deadline.
bool pnn_plan(int F, std::vector<int>& quads, std::vector<int>& colmap, std::vector<int>& sched, std::vector<int>& pro,
              int& KSX, int& KS) {
  if (F < 2 || F > kPMaxF) return false;
  quads.clear();
  for (int i = 0; i + 1 < F; ++i)
    for (int j0 = i + 1; j0 < F; j0 += 4) quads.push_back(i | j0 << 8);
  const int nq = (int)quads.size();
  const int KSP = (nq + 7) / 8;
  quads.resize((size_t)KSP * 8, (F - 1) | (F - 1) << 8);
  KSX = (F + 1) / 2;
  KS = KSX + KSP;
  const int K1 = 16 * F;
  colmap.assign((size_t)KS * 32, -1);
  for (int p = 0; p < K1; ++p) colmap[p] = p;
  for (int q = 0; q < nq; ++q) {
    const int i = quads[q] & 255, j0 = quads[q] >> 8;
    for (int e = 0; e < 4; ++e) {
      const int j = j0 + e;
      if (j < F) colmap[(size_t)KSX * 32 + q * 4 + e] = K1 + i * (2 * F - i - 1) / 2 + (j - i - 1);
    }
  }
  // last ip step reading each field (the fragment of step s is computed during unit KSX + s - 1)
  std::vector<int> last((size_t)F, -1);
  for (int q = 0; q < KSP * 8; ++q) {
    const int s = q / 8, i = quads[q] & 255, j0 = quads[q] >> 8;
    last[i] = std::max(last[i], s);
    for (int e = 0; e < 4; ++e) last[std::min(j0 + e, F - 1)] = std::max(last[std::min(j0 + e, F - 1)], s);
  }
  // next block's pair c: rows at unit t_row(c) of this block's timeline (>= KS: the next block's own unit
  // t_row - KS), ids one unit earlier
  std::vector<int> trow((size_t)KSX), tid((size_t)KSX);
  for (int c = 0; c < KSX; ++c) {
    int ls = last[2 * c];
    if (2 * c + 1 < F) ls = std::max(ls, last[2 * c + 1]);
    int t = KSX + ls;  // step ls's fragment, its last reader, is computed during unit KSX + ls - 1
    if (c > 0) t = std::max(t, trow[c - 1] + 1);
    trow[c] = t;
    tid[c] = t - 1;
    if (t > KS + c - 1) return false;                 // rows must land before the next block's unit c
    if (c >= 4 && tid[c] < trow[c - 4]) return false;  // id slot c & 3 still holds pair c - 4's ids
  }
  sched.assign((size_t)KS, kNone | kNone << 8);
  pro.assign((size_t)KSX, 0);
  for (int c = 0; c < KSX; ++c) {
    const int tr = trow[c] < KS ? trow[c] : trow[c] - KS, ti = tid[c] < KS ? tid[c] : tid[c] - KS;
    if ((sched[tr] & 127) != kNone || ((sched[ti] >> 8) & 127) != kNone) return false;
    sched[tr] = (sched[tr] & ~127) | c;
    sched[ti] = (sched[ti] & ~(127 << 8 | 1 << 15)) | c << 8 | (tid[c] < KS ? 1 << 15 : 0);
    pro[c] = trow[c] < KS ? 2 : (tid[c] < KS ? 1 : 0);
    if (trow[c] >= KS && trow[c] - KS >= c) return false;
  }
  return true;
}

}  // namespace

void pnn_head_release(PnnHead& ph) {
  for (void* q : {(void*)ph.W, (void*)ph.quads, (void*)ph.sched, (void*)ph.pro})
    if (q) (void)hipFree(q);
  ph = PnnHead{};
}

int pnn_head_prepare(hipStream_t s, const float* mats_dev, const DenseLayer& L0, int F, PnnHead& ph) {
  std::vector<int> quads, colmap, sched, pro;
  int KSX = 0, KS = 0;
  if (L0.K1 != 16 * F || L0.Npad != kQN || L0.N > kQN || !pnn_plan(F, quads, colmap, sched, pro, KSX, KS)) {
    pnn_head_release(ph);
    return RMX_OK;  // not eligible: the unfused path runs
  }
  if (!ph.W || ph.F != F || ph.KS != KS) {
    pnn_head_release(ph);
    if (hipMalloc(&ph.W, sizeof(bf16_t) * (size_t)KS * 32 * kQN) != hipSuccess ||
        hipMalloc(&ph.quads, sizeof(int) * quads.size()) != hipSuccess ||
        hipMalloc(&ph.sched, sizeof(int) * (sched.size() + colmap.size())) != hipSuccess ||
        hipMalloc(&ph.pro, sizeof(int) * pro.size()) != hipSuccess) {
      pnn_head_release(ph);
      set_error("out of device memory");
      return RMX_E_NOMEM;
    }
  }
  ph.F = F;
  ph.KSX = KSX;
  ph.KS = KS;
  int* cm = ph.sched + sched.size();  // the column map rides behind the schedule (packing only)
  RMX_HIP(hipMemcpyAsync(ph.quads, quads.data(), sizeof(int) * quads.size(), hipMemcpyHostToDevice, s));
  RMX_HIP(hipMemcpyAsync(ph.sched, sched.data(), sizeof(int) * sched.size(), hipMemcpyHostToDevice, s));
  RMX_HIP(hipMemcpyAsync(cm, colmap.data(), sizeof(int) * colmap.size(), hipMemcpyHostToDevice, s));
  RMX_HIP(hipMemcpyAsync(ph.pro, pro.data(), sizeof(int) * pro.size(), hipMemcpyHostToDevice, s));
  const int64_t tot = (int64_t)KS * 32 * kQN;
  hipLaunchKernelGGL(pnn_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats_dev, L0, cm, KS, ph.W);
  RMX_HIP(hipGetLastError());
  // the host vectors die here: the copies above are pageable, staged before hipMemcpyAsync returns
  RMX_HIP(hipStreamSynchronize(s));
  return RMX_OK;
}

bool pnn_head_usable(const PnnHead& ph, const DenseLayer& L0, int M, int F, int k, bool ids) {
  if (M <= 0 || !ids || k != 16 || !ph.W || ph.F != F || L0.K1 != 16 * F || L0.Npad != kQN || !L0.b) return false;
  // knob "pnn_head": 0 off, 2 always, 1 when the 64-sample row blocks fill every CU
  const int knob = tuning_get("pnn_head", 0);  // (default flipped on once measured on the GPU)
  if (knob == 0) return false;
  if (knob == 2) return true;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  return (M + kPBM - 1) / kPBM >= ncu;
}

int launch_pnn_head(hipStream_t s, const PnnHead& ph, const DenseLayer& L0, int M, int F, const int32_t* ids,
                    const bf16_t* table, bf16_t* H, int ldc) {
  if (M <= 0) return RMX_OK;
  if (!ph.W || ph.F != F || ldc != kQN || !H || !ids || (int64_t)M * F >= (int64_t)1 << 31) {
    set_error("pnn head: not prepared for this model / batch");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipFuncSetAttribute((const void*)pnn_head_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPLds));
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  PnnArgs p{};
  p.M = M;
  p.nblk = (M + kPBM - 1) / kPBM;
  p.F = F;
  p.KSX = ph.KSX;
  p.KS = ph.KS;
  p.ids = ids;
  p.table = table;
  p.W = ph.W;
  p.b = L0.b;
  p.N1 = L0.N;
  p.H = H;
  p.quads = ph.quads;
  p.sched = ph.sched;
  p.pro = ph.pro;
  const int grid = std::min(p.nblk, std::max(ncu, 1));
  hipLaunchKernelGGL(pnn_head_kernel, dim3(grid), dim3(kPThreads), kPLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
