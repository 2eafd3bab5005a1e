// k_small_s3.hip -- DeepFM's whole fp32 tower for small launch batches: one block per 16 or 32 samples,
// all three layers + the FM / first order + the head in one launch, on the split GEMM (gfx950).
//
// The tower (model/encoder/HigherOrderEncoder.scala:34-59: Linear(F k -> 400) + ReLU, 400 -> 400 + ReLU,
// 400 -> 400 + ReLU, Linear(400 -> 1)), the first order (bnn/Scatter.scala:17-36), the FM second order
// (SecondOrderEncoder.scala:19-34) and DeepFM's head (DeepFM.scala:54-80: CAddTable + Sigmoid).
// Why: below ~32 K samples the row-owner kernels (k_head_s3 / k_tail_s3: 128 rows per block) and the
// column-sliced split GEMM (128-row blocks x 2 slices) launch far fewer blocks than the 256 CUs -- at
// B = 4,096 layer 1 ran 64 blocks -- and each layer is its own launch.  Here a block owns RT row tiles of
// 16 samples (B = 4,096 -> 256 blocks of 16) and keeps them on the CU through all three layers: the
// gathered x tile and the activations live in LDS, the 8 waves split the 25 column tiles (wave w: tiles
// w, w + 8, w + 16, w + 24), and each wave streams its own weight fragments (1 KiB contiguous per plane,
// K step and tile) straight from L2 into registers one K step ahead, each fragment feeding the RT row
// tiles -- a fragment is read by exactly one wave of the block, so LDS staging would buy no reuse.  The
// bound is that stream: ~3.6 MB of split planes per block at ~70 GB/s per CU (a K step two ahead
// measured no faster), so a block's time hardly depends on RT.
// Arithmetic: the engine's split products in the engine's order per K step (k_gemm.hpp kPrecS3, operands
// swapped as in k_rowown.hpp), the FM / first order in encoder_k16_kernel<1>'s order (bit-identical).
#include "k_gemm.hpp"

#ifndef RMX_SMALL_DIAG
#define RMX_SMALL_DIAG 0
#endif

namespace rmx {
namespace {

constexpr int kSW = 8;                    // waves
constexpr int kSThreads = kSW * 64;
constexpr int kSN = 416;                  // Npad of the 400-wide layers
constexpr int kSNT = 25;                  // computed column tiles (wave 0: 4, waves 1 .. 7: 3)
static_assert(4 + 7 * 3 == kSNT, "the column split");
constexpr int kSMaxF = 40;
constexpr int kSXS = kSMaxF * 16 + 4;     // x tile row stride (floats): +4 keeps the 16-B reads conflict-free
constexpr int kSHS = kSN + 4;             // activation tile row stride
constexpr int kSTW = 4;                   // max column tiles per wave (wave 0: 4, the others 3)
// RT row tiles of 16 samples per block (kSR samples): each weight fragment loaded feeds RT MFMA row tiles
template <int RT>
constexpr size_t small_lds() {
  return sizeof(float) * (16 * RT * kSXS + 16 * RT * kSHS + kSW * 16 * RT + 3 * kSN + 16 * RT + 16 * RT * kSMaxF) +
         sizeof(int) * 16 * RT * kSMaxF;
}
static_assert(small_lds<2>() <= 160 * 1024, "LDS budget");

struct SmallArgs {
  int M, F;
  const int32_t* ids;     // [M][F]
  const float* table;     // row of id at table + (id << gsh)
  int gsh;
  const float* wtab;      // first-order weight of id at wtab[id << wsh]
  int wsh;
  const bf16_t* W[3];     // split planes [KS_l][3][416][32] of the three layers (DenseLayer::W3)
  const float* b[3];      // [416]
  int KS1;                // K steps of layer 1 (ceil(F / 2)); layers 2 / 3: 13
  OutArgs oa;             // wo [416], bo, beta, out (pre: ignored -- the first order + FM are computed here)
};

// the wave's weight fragments of K step c (tiles w + 8 j, three planes; lane: 16 B of each 1-KiB fragment)
template <int NTW>
__device__ __forceinline__ void s_ldw(const bf16_t* __restrict__ W, int c, int w, int wo, f32x4 (&b)[NTW][3]) {
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      b[j][pl] = *reinterpret_cast<const f32x4*>(W + ((int64_t)(c * 3 + pl) * kSN + 16 * (w + 8 * j)) * 32 + wo);
}

// one layer: acc[j] (column tile w + 8 j) = sum over K steps of W_t x^T on the split planes, x from LDS
// (row stride XS floats); weight fragments of step c + 1 loaded during step c.  bp: on entry step 0's
// fragments (loaded by the caller, ahead of the barriers before the layer); on exit, when Wn is not null,
// the next layer's step 0, loaded during this layer's last step.  PAD (the 400-wide
// layers): the upper half of the last step, columns 400 .. 415, is K padding that no wave writes (25 of
// the 26 tiles are computed) -- read as zeros, as the tails do: its weights are zero, but the LDS there
// holds whatever an earlier workgroup left, and 0 x a leftover NaN / Inf is NaN, which ReLU turns into a
// silently wrong 0 (seen as one wrong row in some blocks, depending on what ran before on the CU)
template <int NTW, int RT, bool PAD, int DG, bool IL>
__device__ __forceinline__ void s_layer(const bf16_t* __restrict__ W, const float* xin, int xs, int KS, int w, int lane,
                                        f32x4 (&acc)[RT][kSTW], f32x4 (&bp)[NTW][3], const bf16_t* __restrict__ Wn) {
  const int g = lane >> 4, r16 = lane & 15;
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int j = 0; j < kSTW; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int wo = r16 * 32 + g * 8;  // lane's element of a fragment
  asm volatile("" : "+v"(wo));
  f32x4 b0[NTW][3], b1[NTW][3];  // (two named buffers: a [2][..] array indexed by c & 1 went to scratch)
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) b0[j][pl] = bp[j][pl];
  int xo = r16 * xs + 4 * g;
  asm volatile("" : "+v"(xo));
  auto step = [&](int c, f32x4 (&cur)[NTW][3], f32x4 (&nxt)[NTW][3]) {
    // the next step's fragments, unconditionally: the next step of this layer, the next layer's step 0, or
    // past the last layer its last step again (unused) -- a load skipped on some path makes the compiler's
    // vmcnt waits count only the loads of the other path, which drained the next step's requests too
    const bool more = c + 1 < KS;
    const bf16_t* __restrict__ Ws = more ? W : (Wn ? Wn : W);
    const int cs = more ? c + 1 : (Wn ? 0 : KS - 1);
    auto ld = [&](int q) {  // fragment q = 3 j + pl of the next step
      if constexpr ((DG & 2) == 0)
        nxt[q / 3][q % 3] =
            *reinterpret_cast<const f32x4*>(Ws + ((int64_t)(cs * 3 + q % 3) * kSN + 16 * (w + 8 * (q / 3))) * 32 + wo);
      else
        nxt[q / 3][q % 3] = cur[q / 3][q % 3] + f32x4{1e-30f, 0.f, 0.f, 0.f};
    };
    if constexpr (!IL) {
#pragma unroll
      for (int q = 0; q < 3 * NTW; ++q) ld(q);
      __builtin_amdgcn_sched_barrier(0);  // (issued before this step's work: the scheduler would sink them)
    }
    bf16x8 ah[RT], am[RT], al[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(xin + xo + 16 * t * xs + 32 * c);
      f32x4 a1 = *reinterpret_cast<const f32x4*>(xin + xo + 16 * t * xs + 32 * c + 16);
      if (PAD && c == KS - 1) a1 = f32x4{0.f, 0.f, 0.f, 0.f};
      split3(a0, a1, ah[t], am[t], al[t]);
    }
    // the six products in the engine's order, each over all the wave's (row tile, column tile) pairs;
    // IL: two of the next step's fragment loads after each product group, so a wave's vector-memory issue
    // is spread over its MFMA stream instead of stalling it in one burst at the step head
#pragma unroll
    for (int pr = 0; pr < 6; ++pr) {
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const bf16x8 bh = __builtin_bit_cast(bf16x8, cur[j][0]);
        const bf16x8 bm = __builtin_bit_cast(bf16x8, cur[j][1]);
        const bf16x8 bl = __builtin_bit_cast(bf16x8, cur[j][2]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
          if constexpr ((DG & 1) != 0) {
            if (pr == 0) acc[t][j] += cur[j][0] + __builtin_bit_cast(f32x4, ah[t]);
            continue;
          }
          const bf16x8 wa = pr == 0 || pr == 4 ? bm : (pr == 2 ? bl : bh);
          const bf16x8 xa = pr == 1 ? al[t] : (pr == 0 || pr == 3 ? am[t] : ah[t]);
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, xa, acc[t][j], 0, 0, 0);
        }
      }
      if constexpr (IL) {
        if (2 * pr < 3 * NTW) ld(2 * pr);
        if (2 * pr + 1 < 3 * NTW) ld(2 * pr + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
#pragma unroll 1
  for (int c = 0; c < KS; c += 2) {
    step(c, b0, b1);
    if (c + 1 < KS) step(c + 1, b1, b0);
  }
  // the last step (KS - 1) loaded the next layer's step 0 into b1 when it was an even step, else into b0
  const bool odd = (KS & 1) != 0;
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) bp[j][pl] = odd ? b1[j][pl] : b0[j][pl];
}

// ReLU(acc + b) of the wave's tiles into the activation tile (lane: row r16, columns 16 t + 4 g .. + 3)
template <int NTW, int RT>
__device__ __forceinline__ void s_store_h(const f32x4 (&acc)[RT][kSTW], const float* bl, float* h, int w, int lane) {
  const int g = lane >> 4, r16 = lane & 15;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int n0 = 16 * (w + 8 * j) + 4 * g;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + n0);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      f32x4 v = acc[t][j] + bb;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
      *reinterpret_cast<f32x4*>(h + (16 * t + r16) * kSHS + n0) = v;
    }
  }
}

// the whole block (every wave runs it, NTW = the wave's tile count): layer 1's first weight fragments are
// requested before the prologue (ids, the gathered rows, the first-order weights, FM), so their latency
// overlaps it; each layer's last K step requests the next layer's first fragments.
template <int NTW, int RT, int DG, bool IL>
__device__ void s_wave(const SmallArgs& p, float* ssmem, int tid, int w, int lane) {
  constexpr int kSR = 16 * RT;
  float* x = ssmem;                       // [kSR][kSXS] gathered rows; later layer 2's output
  float* h = x + kSR * kSXS;              // [kSR][kSHS] layer 1's output
  float* red = h + kSR * kSHS;            // [8 waves][kSR] partial logits
  float* prm = red + kSW * kSR;           // b1 | b2 | b3
  float* fmv = prm + 3 * kSN;             // [kSR] first order + FM (y1 + y2) per sample
  float* swt = fmv + kSR;                 // [kSR][F] first-order weights of the ids
  int* sid = reinterpret_cast<int*>(swt + kSR * kSMaxF);  // [kSR][F] ids
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = blockIdx.x * kSR, F = p.F;
  f32x4 bp[NTW][3];
  {
    int wo = r16 * 32 + g * 8;
    asm volatile("" : "+v"(wo));
    s_ldw<NTW>(p.W[0], 0, w, wo, bp);
  }
  // the prologue's loads are issued a whole phase at a time (fixed trip counts, unrolled, every load
  // unconditional: a slot past the data reads the zero / -1 words), so each phase waits one memory latency,
  // not one per loop iteration: the biases and the ids, then the gathered rows and the first-order weights
  // (both from the ids)
  const float* zero16 = g_rmx_zero16;
  const int* neg1 = g_rmx_neg1;
  {
    constexpr int NP = (3 * kSN + kSThreads - 1) / kSThreads, NI = (kSR * kSMaxF + kSThreads - 1) / kSThreads;
    float pv[NP];
    int iv[NI];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int i = tid + u * kSThreads, a = i / kSN, n = i - a * kSN;
      const float* src = a == 0 ? p.b[0] : (a == 1 ? p.b[1] : p.b[2]);  // (no dynamic index into the kernel args)
      pv[u] = *((i < 3 * kSN && src) ? src + n : zero16);
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + u * kSThreads, r = i / F, m = m0 + r;
      const bool ok = i < kSR * F && m < p.M;
      // (ids == nullptr: the L-A path's staged rows, id = m F + f)
      iv[u] = p.ids ? *(ok ? p.ids + (int64_t)m * F + (i - r * F) : neg1) : (ok ? m * F + (i - r * F) : -1);
    }
#pragma unroll
    for (int u = 0; u < NP; ++u)
      if (tid + u * kSThreads < 3 * kSN) prm[tid + u * kSThreads] = pv[u];
#pragma unroll
    for (int u = 0; u < NI; ++u)
      if (tid + u * kSThreads < kSR * F) sid[tid + u * kSThreads] = iv[u];
  }
  __syncthreads();
  // the gathered rows: x[r][16 f + j] (fields past F and rows past M: zero); the first-order weights
  {
    constexpr int NX = (kSR * kSMaxF * 4 + kSThreads - 1) / kSThreads, NW = (kSR * kSMaxF + kSThreads - 1) / kSThreads;
    float4 xv[NX];
    float wv[NW];
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int i = tid + u * kSThreads;
      const int r = i / (kSMaxF * 4), rest = i - r * (kSMaxF * 4), f = rest >> 2, q = rest & 3;
      const int id = i < kSR * kSMaxF * 4 && f < F ? sid[r * F + f] : -1;
      xv[u] = *reinterpret_cast<const float4*>((DG & 4) == 0 && id >= 0 ? p.table + ((int64_t)id << p.gsh) + 4 * q
                                                                        : zero16);
    }
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int i = tid + u * kSThreads;
      const int id = i < kSR * F ? sid[i] : -1;
      wv[u] = *((DG & 4) == 0 && id >= 0 ? p.wtab + ((int64_t)id << p.wsh) : zero16);
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int i = tid + u * kSThreads;
      const int r = i / (kSMaxF * 4), rest = i - r * (kSMaxF * 4), f = rest >> 2, q = rest & 3;
      if (i < kSR * kSMaxF * 4) *reinterpret_cast<float4*>(x + r * kSXS + 16 * f + 4 * q) = xv[u];
    }
#pragma unroll
    for (int u = 0; u < NW; ++u)
      if (tid + u * kSThreads < kSR * F) swt[tid + u * kSThreads] = wv[u];
  }
  __syncthreads();
  // first order + FM of sample r (16 lanes per sample, lane j of the group: column j; wave w takes samples
  // 4 w .. 4 w + 3, then + 32), in encoder_k16_kernel<1>'s order: s_j, q_j over the fields in order,
  // a = sum_j (s_j^2 - q_j) in j order, y1 = the first-order weights summed in field order
  {
#pragma clang fp contract(off)
    for (int rr = 4 * w; rr < kSR; rr += 4 * kSW) {
      const int r = rr + (lane >> 4), j = lane & 15;
      float s = 0.f, q = 0.f;
      for (int f = 0; f < F; ++f) {
        const float e = x[r * kSXS + 16 * f + j];
        s = s + e;
        q = q + e * e;
      }
      const float d = s * s - q;
      float a = 0.f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) a += __shfl(d, (lane & 48) + jj);
      float y1 = 0.f;
      for (int f = 0; f < F; ++f) y1 += swt[r * F + f];
      if (j == 0) fmv[r] = y1 + 0.5f * (a / 16.0f);
    }
  }
  __syncthreads();

  f32x4 acc[RT][kSTW];
  // layer 1: x tile (row stride kSXS) -> h
  s_layer<NTW, RT, false, DG, IL>(p.W[0], x, kSXS, p.KS1, w, lane, acc, bp, p.W[1]);  // (x: every column written)
  s_store_h<NTW, RT>(acc, prm, h, w, lane);
  __syncthreads();
  // layer 2: h -> the x region (stride kSHS)
  s_layer<NTW, RT, true, DG, IL>(p.W[1], h, kSHS, 13, w, lane, acc, bp, p.W[2]);
  __syncthreads();  // every wave has read h ... (the x region is free since layer 1)
  s_store_h<NTW, RT>(acc, prm + kSN, x, w, lane);
  __syncthreads();
  // layer 3 + the output dot over the wave's columns
  s_layer<NTW, RT, true, DG, IL>(p.W[2], x, kSHS, 13, w, lane, acc, bp, nullptr);
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n0 = 16 * (w + 8 * j) + 4 * g;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + 2 * kSN + n0);
      const f32x4 wv = *reinterpret_cast<const f32x4*>(p.oa.wo + n0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[t][j][r] + bb[r];
        v = v > 0.f ? v : 0.f;
        part += v * wv[r];
      }
    }
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    if (g == 0) red[w * kSR + 16 * t + r16] = part;
  }
  __syncthreads();
  if (tid < kSR) {
    const int m = m0 + tid;
    if (m < p.M) {
      float y = red[tid];
#pragma unroll
      for (int q = 1; q < kSW; ++q) y += red[q * kSR + tid];
      const OutArgs& oa = p.oa;
      if (oa.has_bo) y = y + oa.bo;
      float t = fmv[tid] + y;  // pre (first order + FM) + the tower's logit, out_finish_kernel's order
      t = t + oa.beta;
      oa.out[m] = 1.0f / (1.0f + expf(-t));
    }
  }
}

template <int RT, int DG, bool IL>
__global__ __launch_bounds__(kSThreads, 1) void tower_small_s3_kernel(SmallArgs p) {
  extern __shared__ __attribute__((aligned(16))) float ssmem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (w == 0)
    s_wave<4, RT, DG, IL>(p, ssmem, tid, w, lane);
  else
    s_wave<3, RT, DG, IL>(p, ssmem, tid, w, lane);
}

}  // namespace

bool tower_small_s3_usable(const rmx_model& m, int M, int F, int k, bool ids) {
  if (M <= 0 || !ids || k != 16 || F < 1 || F > kSMaxF || m.type != RMX_MODEL_DEEPFM || m.layers.size() != 3 ||
      !f32_split_enabled() || m.precision != kF32)
    return false;
  for (int l = 0; l < 3; ++l) {
    const DenseLayer& L = m.layers[l];
    if (!L.W3 || L.W16 || L.N != 400 || L.Npad != kSN || L.N1 >= 0 || L.bias_mode != 1 || L.K1 >= 0) return false;
    if (L.K != (l == 0 ? 16 * F : 400)) return false;
  }
  // knob "s3_small": 0 off, 2 always, 1 (default) up to one 16-sample block per CU
  // (default 1 since measured: DeepFM B = 4,096 40.8 -> 50.1 M examples/s, profiles/r04/ab_round4_first.txt)
  const int knob = tuning_get("s3_small", 1);
  if (knob == 0) return false;
  if (knob == 2) return true;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  // one round of 16- or 32-sample blocks (B <= 8,192 on 256 CUs): every block streams all three layers'
  // weights, so a second round costs a whole round again (B = 16,384: 53 M examples/s, against ~156 M on
  // the row-owner head + tail's half blocks, profiles/r04/grid_summary.txt)
  return M <= tuning_get("s3_small_max", 32 * ncu);
}

int launch_tower_small_s3(hipStream_t s, const rmx_model& m, int M, int F, const int32_t* ids, const float* table,
                          int ld, const float* wtab, int wld, const OutArgs& oa) {
  if (M <= 0) return RMX_OK;
  const int l = ld > 0 ? ld : 16, wl = wld > 0 ? wld : 1;
  if ((l & (l - 1)) || l < 16 || (wl & (wl - 1)) || !oa.wo || !oa.out) {
    set_error("fp32 small tower: table / weight strides must be powers of two, and an output head");
    return RMX_E_INVALID;
  }
  // knob "s3_small_rt": row tiles of 16 samples per block, 1 or 2; 0 (default) = 1 while 16-sample blocks
  // fit one round on the CUs, else 2.  Each CU streams the whole tower's split weights at ~70 GB/s whatever
  // its row count, and a second row tile costs only its MFMAs: B = 8,192 one round of 32-sample blocks
  // 0.072 ms (111 M examples/s) against the head + tail's 0.102 ms; B = 4,096 16-sample blocks 0.0645 vs
  // 0.071 ms (profiles/r04/ab_small_rt.txt)
  int rt = tuning_get("s3_small_rt", 0);
  if (rt != 1 && rt != 2) {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
    rt = M <= 16 * ncu ? 1 : 2;
  }
  SmallArgs p{};
  p.M = M;
  p.F = F;
  p.ids = ids;
  p.table = table;
  p.gsh = __builtin_ctz((unsigned)l);
  p.wtab = wtab;
  p.wsh = __builtin_ctz((unsigned)wl);
  for (int i = 0; i < 3; ++i) {
    p.W[i] = m.layers[i].W3;
    p.b[i] = m.layers[i].b;
  }
  p.KS1 = (F + 1) / 2;
  p.oa = oa;
  // (IL = false: the next step's loads at the step head, measured 0.0704 vs 0.069 ms at B = 8,192 --
  // profiles/r05/ab_small_il_wgrad16.txt; DG: timing probes, built only with RMX_SMALL_DIAG, results wrong)
  const void* fn = rt == 2 ? (const void*)tower_small_s3_kernel<2, 0, true> : (const void*)tower_small_s3_kernel<1, 0, true>;
#if RMX_SMALL_DIAG
  const int dg = tuning_get("s3_small_diag", 0);  // 1 no MFMA, 2 no weight loads, 4 no gather (tools/probe_small.py)
#define RMX_DG(V) \
  if (rt == 1 && dg == V) fn = (const void*)tower_small_s3_kernel<1, V, true>;
  RMX_DG(1) RMX_DG(2) RMX_DG(3) RMX_DG(4) RMX_DG(7)
#undef RMX_DG
#endif
  const size_t lds = rt == 2 ? small_lds<2>() : small_lds<1>();
  RMX_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* args[] = {&p};
  RMX_HIP(hipLaunchKernel(fn, dim3((M + 16 * rt - 1) / (16 * rt)), dim3(kSThreads), args, lds, s));
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
