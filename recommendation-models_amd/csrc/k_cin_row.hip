// k_cin_row.hip -- xDeepFM's whole CIN stack in one persistent row-owner kernel (gfx950), BASELINE.json
// configs[2] (fp32).
//
// CIN layer l (xdeepfm/CINEncoder.scala:135-176): for each sample and embedding coordinate t,
//   z_l[t][f, h] = x0[f][t] * u_{l-1}[t][h]          (u_0 = x0)
//   u_l[t][n]    = ReLU(sum_{f,h} z_l[t][f, h] C_l[n][f, h] + b_l[n])
// and the pooled maps feed the output Linear: rowdot[b k + t] = sum_l sum_n u_l[t][n] wo_l[n]
// (out_finish / the tower head sums the k rows of a sample).
//
// The per-layer engine (k_gemm.hpp, kPrecS3) runs each layer as one GEMM over M = B k rows and writes u_l
// (B k x 208 fp32) to HBM for the next layer.  Here a wave owns ONE sample (its k = 16 rows) for the whole
// stack, and nothing but the gathered x0 rows and rowdot touches HBM:
//   * the MFMA runs with operands swapped (D = C_l z^T, v_mfma_f32_16x16x32_bf16, weights as A), so lane
//     (t, g) holds u_l[t][16 j + 4 g + q] for column tile j -- exactly the h values lane group g needs in
//     the next layer's K chunks (h-chunk j, element 4 g + q: the split engine's chunk convention).  So u_l
//     stays in 13 x 4 registers and z is formed in registers: x0[f][t] (the wave's LDS image) times them;
//   * the K order is the engine's chunk map (cin_chunk_map: h-chunk major, fields minor; layer 1 folded
//     to h <= f; a last h-chunk with <= 8 live maps carries two fields per chunk), padded to an even
//     number of chunks per h-chunk so a 32-wide K step never straddles two h-chunks (the h-chunk loop is
//     unrolled, so the u registers it reads are static).  Layer 1 runs 34 K steps, layers 2 and 3 250
//     each at F = 39, H = 200 (the engine: 31 and 254);
//   * the split arithmetic is the engine's: z = hi + mid + lo (bf16), C_l pre-split into 3 planes, six
//     products per K step in the engine's order (k_rowown.hpp q_unit);
//   * the weights of all layers stream through the 3-slot LDS ring of k_rowown.hpp (one unit = one K step x
//     13 tiles x 3 planes = 39 KiB; 5 DMAs per wave), one barrier per unit, continuing across samples;
//   * the next sample's ids and x0 rows are gathered (LDS DMA) into the wave's second image during the
//     current sample's units 3 and 5.
// LDS: 3 x 39,936 + 8 x (2 x 2,560 + 256) = 162,816 B.
#include "k_rowown.hpp"
#include "rmx_models.hpp"

#include <vector>

namespace rmx {
namespace {
using namespace rowown;

constexpr int kCN = 208;                     // Npad of a CIN layer
constexpr int kCT = 13;                      // column tiles (= h-chunks of the next layer)
constexpr int kCImg = 40 * 64;               // per wave x0 image: [40 fields][16 t] fp32
constexpr int kCIds = 64 * 4;                // per wave id slot
constexpr int kCWave = 2 * kCImg + kCIds;
constexpr size_t kCLds = (size_t)kQSlots * kQUnit + (size_t)kQW * kCWave;
static_assert(kCLds <= 160 * 1024, "LDS budget");
static_assert(3 * kCT * 1024 == kQUnit, "a CIN unit is a k_rowown unit");
constexpr int kCIdUnit = 3, kCRowUnit = 5;  // units of a sample that gather the next sample's ids / rows
constexpr int kCMaxL = 4;

struct CinRowArgs {
  int B, ngrp, F, L, S;            // samples, groups of 8, fields, layers, units per sample
  const int32_t* ids;              // [B][F]
  const float* table;              // [rows][16] fp32
  const bf16_t* W;                 // [S][3][208][32]: every layer's units in order
  const float* bw;                 // [L][2][208]: b_l | wo_l
  float* rowdot;                   // [B * 16]
  int nu1[4], f01[4], pr1[4];      // layer 1 per h-chunk: units, first field, two-fields-per-chunk
  int nu2[kCT], f02[kCT], pr2[kCT];  // layers >= 2
};

// ids of sample b into the wave's id slot (lane L < F: field L; else -1)
__device__ __forceinline__ void c_id_dma(const CinRowArgs& p, char* wl, int b, int lane) {
  const bool ok = b < p.B && lane < p.F;
  const int32_t* src = ok ? p.ids + (int64_t)b * p.F + lane : g_rmx_neg1;
  lds_dma<4>(src, wl + 2 * kCImg);
}
// x0 rows of the sample whose ids are in the slot into image `img` (3 DMAs: 16 rows of 64 B each, lane L
// = row 16 i + (L >> 2), 16-B part L & 3; the third only rows 32 .. 39)
__device__ __forceinline__ void c_row_dma(const CinRowArgs& p, char* wl, int img, int lane) {
  const int* ids = reinterpret_cast<const int*>(wl + 2 * kCImg);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    int rr = 16 * i + (lane >> 2), part = lane & 3;
    asm volatile("" : "+v"(rr), "+v"(part));
    const int id = ids[rr];
    const float* src = id >= 0 ? p.table + ((int64_t)id << 4) + 4 * part : g_rmx_zero16;
    if (i < 2 || lane < 32) lds_dma<16>(src, wl + img * kCImg + i * 1024);
  }
}

// One CIN layer over the wave's sample.  u: the previous layer's maps (lane (t, g): h = 16 j + 4 g + q in
// u[j]); acc: this layer's pre-activation.  NHC h-chunks, per chunk hc: nu[hc] units of two chunks (plain:
// fields f0 + 2 v, f0 + 2 v + 1; pair: fields f0 + 4 v + (g >> 1) and + 2, maps 16 hc + 4 (g & 1) ..).
template <int NHC, bool FIRST>
__device__ __forceinline__ void c_layer(const CinRowArgs& p, char* lds, const float* x0, const f32x4 (&u)[kCT],
                                        f32x4 (&acc)[kCT], int& slot, int& us, int64_t& U, int w, int lane, int lo,
                                        int fb, char* wl, int bnext, int imgn) {
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < kCT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int hc = 0; hc < NHC; ++hc) {
    const int n = FIRST ? p.nu1[hc] : p.nu2[hc], fs = FIRST ? p.f01[hc] : p.f02[hc];
    const int pair = FIRST ? p.pr1[hc] : p.pr2[hc];
    // a pair chunk's lane groups 2, 3 take the maps of groups 0, 1 (lane - 32)
    f32x4 uv = u[hc];
    {
      f32x4 us2;
#pragma unroll
      for (int q = 0; q < 4; ++q) us2[q] = __shfl(uv[q], lane & 31);
      if (pair) uv = us2;
    }
    const int fstep = pair ? 4 : 2, fadd = pair ? (g >> 1) : 0, fsec = pair ? 2 : 1;
#pragma unroll 1
    for (int v = 0; v < n; ++v) {
      q_enter<5>();
      int fa = fs + fstep * v + fadd, fbb = fa + fsec;
      fa = fa < 39 ? fa : 39;  // pad chunks: any finite x0 (their weights are zero)
      fbb = fbb < 39 ? fbb : 39;
      const float xa = x0[fa * 16], xb = x0[fbb * 16];
      bf16x8 ah, am, al;
      split3(xa * uv, xb * uv, ah, am, al);
      const int64_t u2 = U + 2 < p.S ? U + 2 : U + 2 - p.S;
      const int dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kCT, 0, kCT, 2, kCN>(lds + slot * kQUnit, fb, ah, am, al, acc, p.W + u2 * (3 * kCN * 32), lds, dslot, w,
                                  lo);
      slot = q_next(slot);
      // the next sample's ids, then (two units later: they have landed) its rows -- after the unit's
      // weight DMAs, so the next unit's vmcnt(5) still covers this unit's ring slot
      if (us == kCIdUnit) c_id_dma(p, wl, bnext, lane);
      if (us == kCRowUnit) c_row_dma(p, wl, imgn, lane);
      ++us;
      U = U + 1 < p.S ? U + 1 : 0;
    }
  }
}

template <int NHC1>
__global__ __launch_bounds__(kQThreads, 1) void cin_row_kernel(CinRowArgs p) {
  extern __shared__ __attribute__((aligned(16))) char csmem[];
  char* lds = csmem;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, t16 = lane & 15;
  char* wl = csmem + kQSlots * kQUnit + w * kCWave;
  const int nit = (int)blockIdx.x < p.ngrp ? (p.ngrp - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  int lo = (lane >> 2) * 32 + swz_slot(lane >> 2, lane & 3) * 8;
  asm volatile("" : "+v"(lo));
  const int fb = q_fbase(lane);

  // prologue: the first sample's x0 into image 0, units 0 and 1 of the ring
  c_id_dma(p, wl, blockIdx.x * kQW + w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  c_row_dma(p, wl, 0, lane);
  if (nit > 0) {
#pragma unroll
    for (int q = 0; q < kQQ; ++q) q_dma<kCN>(p.W, lds, 0, w, q, lo);
#pragma unroll
    for (int q = 0; q < kQQ; ++q) q_dma<kCN>(p.W + 3 * kCN * 32, lds, 1, w, q, lo);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int slot = 0;
  int64_t U = 0;
  for (int it = 0; it < nit; ++it) {
    const int grp = blockIdx.x + it * gridDim.x;
    const int b = grp * kQW + w, bnext = (grp + gridDim.x) * kQW + w;
    const int img = it & 1;
    const float* x0 = reinterpret_cast<const float*>(wl + img * kCImg) + t16;  // x0[f][t] at x0[16 f]
    int us = 0;
    float part = 0.f;
    f32x4 u[kCT], acc[kCT];
    // u_0 = x0: lane (t, g) holds x0[16 j + 4 g + q][t]
#pragma unroll
    for (int j = 0; j < kCT; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int h = 16 * j + 4 * g + q;
        u[j][q] = (j < NHC1 && h < p.F) ? x0[(h < 39 ? h : 39) * 16] : 0.f;
      }
    }
    for (int l = 0; l < p.L; ++l) {
      if (l == 0)
        c_layer<NHC1, true>(p, lds, x0, u, acc, slot, us, U, w, lane, lo, fb, wl, bnext, img ^ 1);
      else
        c_layer<kCT, false>(p, lds, x0, u, acc, slot, us, U, w, lane, lo, fb, wl, bnext, img ^ 1);
      // u_l = ReLU(acc + b_l); the pooled output dot
      __builtin_amdgcn_sched_barrier(0);
      const float* bl = p.bw + (int64_t)l * 2 * kCN;
      int g4 = 4 * g;
      asm volatile("" : "+v"(g4));
#pragma unroll
      for (int j = 0; j < kCT; ++j) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 16 * j + g4);
        const f32x4 wv = *reinterpret_cast<const f32x4*>(bl + kCN + 16 * j + g4);
        u[j] = relu4(acc[j] + bb);
#pragma unroll
        for (int q = 0; q < 4; ++q) part += u[j][q] * wv[q];
      }
    }
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    if (g == 0 && b < p.B) p.rowdot[(int64_t)b * 16 + t16] = part;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// C_l (H x F*Hp) -> fp32 [nc][208][16] in the padded chunk order (k_gemm.hip pack_cin_map_kernel's
// element convention; a pad entry has f = F: zero weights)
__global__ void cin_row_pack_kernel(const float* __restrict__ C, int F, int Hp, int H, int tri,
                                    const int* __restrict__ cmap, int64_t tot, float* __restrict__ Wm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int e = (int)(i & 15), g = e >> 2, q = e & 3;
  const int64_t rest = i >> 4;
  const int n = (int)(rest % kCN);
  const int c = (int)(rest / kCN);
  const int ent = cmap[c];
  const int pr = (ent >> 30) & 1, hc = (ent >> 16) & 0x3fff;
  const int f = (ent & 0xffff) + (pr ? g >> 1 : 0);
  const int h = 16 * hc + (pr ? (g & 1) * 4 : g * 4) + q;
  float v = 0.f;
  if (n < H && f < F && h < Hp) {
    const float* Cn = C + (int64_t)n * F * Hp;
    if (!tri)
      v = Cn[(int64_t)f * Hp + h];
    else if (h < f)
      v = Cn[(int64_t)f * Hp + h] + Cn[(int64_t)h * Hp + f];
    else if (h == f)
      v = Cn[(int64_t)f * Hp + f];
  }
  Wm[i] = v;
}

// the padded chunk map of one layer and its per-h-chunk schedule
void cin_row_map(int F, int Hp, bool tri, std::vector<int>& map, int* nu, int* f0, int* pr) {
  map.clear();
  const int nhc = (Hp + 15) / 16;
  for (int hc = 0; hc < nhc; ++hc) {
    const bool pair = Hp - 16 * hc <= 8;
    const int start = tri ? 16 * hc : 0;
    int cnt = 0;
    for (int f = start; f < F; f += pair ? 2 : 1, ++cnt) map.push_back(f | hc << 16 | (pair ? 1 << 30 : 0));
    if (cnt & 1) {
      map.push_back(F | hc << 16 | (pair ? 1 << 30 : 0));  // pad chunk: f = F, zero weights
      ++cnt;
    }
    nu[hc] = cnt / 2;
    f0[hc] = start;
    pr[hc] = pair ? 1 : 0;
  }
}

}  // namespace

void cin_row_release(CinRow& cr) {
  if (cr.W) (void)hipFree(cr.W);
  if (cr.bw) (void)hipFree(cr.bw);
  cr = CinRow{};
}

int cin_row_prepare(hipStream_t s, const float* mats_dev, const rmx_model& m, CinRow& cr) {
  const int F = m.F, L = (int)m.cin_layers.size();
  bool ok = m.k == 16 && F >= 2 && F <= 40 && L >= 1 && L <= kCMaxL;
  for (int l = 0; ok && l < L; ++l) {
    const CinLayer& c = m.cin_layers[l];
    ok = c.Npad == kCN && c.H <= kCN && c.b && c.wo && c.Hp == (l == 0 ? F : m.cin_layers[l - 1].H) &&
         (l == 0 || c.H == m.cin_layers[0].H);
  }
  if (!ok) {
    cin_row_release(cr);
    return RMX_OK;  // the per-layer engine runs
  }
  std::vector<std::vector<int>> maps((size_t)L);
  int nu[kCMaxL][kCT] = {}, f0[kCMaxL][kCT] = {}, pr[kCMaxL][kCT] = {};
  int S = 0;
  for (int l = 0; l < L; ++l) {
    const CinLayer& c = m.cin_layers[l];
    cin_row_map(F, c.Hp, l == 0, maps[l], nu[l], f0[l], pr[l]);
    S += (int)maps[l].size() / 2;
  }
  if (cr.W && cr.S != S) cin_row_release(cr);
  if (!cr.W) {
    if (hipMalloc(&cr.W, sizeof(bf16_t) * (size_t)S * 3 * kCN * 32) != hipSuccess ||
        hipMalloc(&cr.bw, sizeof(float) * (size_t)L * 2 * kCN) != hipSuccess) {
      cin_row_release(cr);
      set_error("out of device memory");
      return RMX_E_NOMEM;
    }
  }
  cr.S = S;
  cr.L = L;
  cr.nhc1 = (F + 15) / 16;
  for (int hc = 0; hc < 4; ++hc) {
    cr.nu1[hc] = nu[0][hc];
    cr.f01[hc] = f0[0][hc];
    cr.pr1[hc] = pr[0][hc];
  }
  for (int hc = 0; hc < kCT; ++hc) {
    cr.nu2[hc] = L > 1 ? nu[1][hc] : 0;
    cr.f02[hc] = L > 1 ? f0[1][hc] : 0;
    cr.pr2[hc] = L > 1 ? pr[1][hc] : 0;
  }
  int64_t off = 0;
  for (int l = 0; l < L; ++l) {
    const CinLayer& c = m.cin_layers[l];
    const int nc = (int)maps[l].size();
    int* dmap = nullptr;
    float* Wm = nullptr;
    if (hipMalloc(&dmap, sizeof(int) * nc) != hipSuccess ||
        hipMalloc(&Wm, sizeof(float) * (size_t)nc * kCN * 16) != hipSuccess) {
      if (dmap) (void)hipFree(dmap);
      cin_row_release(cr);
      set_error("out of device memory");
      return RMX_E_NOMEM;
    }
    int st = RMX_OK;
    if (hipMemcpyAsync(dmap, maps[l].data(), sizeof(int) * nc, hipMemcpyHostToDevice, s) != hipSuccess) st = RMX_E_HIP;
    const int64_t tot = (int64_t)nc * kCN * 16;
    if (!st) {
      hipLaunchKernelGGL(cin_row_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats_dev + c.w_off,
                         F, c.Hp, c.H, l == 0 ? 1 : 0, dmap, tot, Wm);
      if (hipGetLastError() != hipSuccess) st = RMX_E_HIP;
    }
    if (!st) st = launch_pack_split3(s, Wm, nc, kCN, cr.W + off * 3 * kCN * 32);
    if (!st && (hipMemcpyAsync(cr.bw + (int64_t)l * 2 * kCN, c.b, sizeof(float) * kCN, hipMemcpyDeviceToDevice, s) !=
                    hipSuccess ||
                hipMemcpyAsync(cr.bw + (int64_t)l * 2 * kCN + kCN, c.wo, sizeof(float) * kCN,
                               hipMemcpyDeviceToDevice, s) != hipSuccess))
      st = RMX_E_HIP;
    // the temporaries die after the stream drains (the host map vector is pageable: staged by now)
    (void)hipStreamSynchronize(s);
    (void)hipFree(dmap);
    (void)hipFree(Wm);
    if (st) {
      cin_row_release(cr);
      set_error("cin row: packing failed");
      return st;
    }
    off += nc / 2;
  }
  return RMX_OK;
}

bool cin_row_usable(const CinRow& cr, const rmx_model& m, int B, bool ids) {
  if (B <= 0 || !ids || !cr.W || cr.L != (int)m.cin_layers.size() || m.k != 16 || !f32_split_enabled()) return false;
  // knob "cin_row": 0 off, 2 always, 1 when the groups of 8 samples fill every CU at least once (default
  // flipped on once measured on the GPU)
  const int knob = tuning_get("cin_row", 0);
  if (knob == 0) return false;
  if (knob == 2) return true;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  return (B + kQW - 1) / kQW >= ncu;
}

int launch_cin_row(hipStream_t s, const CinRow& cr, const rmx_model& m, int B, const int32_t* ids, const float* table,
                   float* rowdot) {
  if (B <= 0) return RMX_OK;
  if (!cr.W || !ids || !table || !rowdot || m.k != 16 || m.F > 40 || cr.nhc1 < 1 || cr.nhc1 > 3) {
    set_error("cin row: not prepared for this model");
    return RMX_E_INVALID;
  }
  CinRowArgs p{};
  p.B = B;
  p.ngrp = (B + kQW - 1) / kQW;
  p.F = m.F;
  p.L = cr.L;
  p.S = cr.S;
  p.ids = ids;
  p.table = table;
  p.W = cr.W;
  p.bw = cr.bw;
  p.rowdot = rowdot;
  for (int i = 0; i < 4; ++i) {
    p.nu1[i] = cr.nu1[i];
    p.f01[i] = cr.f01[i];
    p.pr1[i] = cr.pr1[i];
  }
  for (int i = 0; i < kCT; ++i) {
    p.nu2[i] = cr.nu2[i];
    p.f02[i] = cr.f02[i];
    p.pr2[i] = cr.pr2[i];
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = std::min(p.ngrp, std::max(ncu, 1));
#define RMX_CIN_ROW(N)                                                                                             \
  RMX_HIP(hipFuncSetAttribute((const void*)cin_row_kernel<N>, hipFuncAttributeMaxDynamicSharedMemorySize,          \
                              (int)kCLds));                                                                        \
  hipLaunchKernelGGL(cin_row_kernel<N>, dim3(grid), dim3(kQThreads), kCLds, s, p);
  if (cr.nhc1 == 1) {
    RMX_CIN_ROW(1)
  } else if (cr.nhc1 == 2) {
    RMX_CIN_ROW(2)
  } else {
    RMX_CIN_ROW(3)
  }
#undef RMX_CIN_ROW
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
