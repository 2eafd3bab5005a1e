// k_gemm.hip -- the fp32 MFMA GEMM engine behind the tower layers and the xDeepFM CIN (gfx950).
//
// Tower layer: BigDL Linear + ReLU chain, model/encoder/HigherOrderEncoder.scala:34-59
// (Linear(in->out, W: out x in, y = b + x W^T) + ReLU per fcDim, then Linear(->1)) and the
// output heads of DeepFM.scala:130-134 / XDeepFM / DCN / PNN (CAddTable + Sigmoid).
// CIN layer: model/xdeepfm/CINEncoder.scala:36-58, 105-176 (+ SURVEY.md Appendix A for L > 1):
//   x0[b,j,f] = e[b,f,j]; z[f*Hp + h] = x0[b,j,f] * u_{l-1}[b,j,h]  (MM(transB = true), :152)
//   u_l[b,j,:] = ReLU(c_l + C_l z)                                   (Linear + ReLU, :154-155)
// a GEMM with M = B*k rows (b, j), K = F * Hp, N = H whose A operand is generated in registers
// (the reference materialises z: B*k x F*Hp floats, 2 GB per layer at B = 4096), and whose
// epilogue folds the output Linear in: rowdot[b*k + j] (+)= sum_h u_l[b,j,h] * W_out[slice_l + h]
// (sum_j sum_h == sum_h sum_j: the pooled pi_l . W_out, :159-176).
//
// All on v_mfma_f32_16x16x4_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD = the chip's fp32 peak).
// Block = WM waves stacked on M; a wave owns MT*16 rows x all NT*16 columns of the block
// (MT*NT accumulator tiles).  WM is a multiple of 4, so every SIMD carries the same number of
// waves and the one barrier per K stage never waits on an overloaded SIMD.  K is consumed in
// 16-wide chunks; inside a chunk lane group g = lane>>4 owns k = 4g..4g+3, so one ds_read_b128
// per fragment feeds the 4 k-steps of the chunk.  LDS tiles are [rows][16] fp32 with a slot
// XOR-swizzle that keeps the 16-row fragment reads conflict-free for all four ds_read_b128 lane
// groups.  A stage holds BKC chunks; the next stage's global loads are issued before the MFMAs
// of the current one and written to the idle LDS buffer after them (one barrier per stage).
// A operand producers:
//   kDenseA     activations of the previous layer, staged through LDS;
//   kGatherK16  / kGatherAny: first layer, rows gathered straight from the embedding table
//               (ids staged in LDS; x = Reshape(B, F*k) is never materialised);
//   kCinOuter   CIN: a = x0[row][f] * u[row][h-chunk], computed in registers (x0 tile in LDS,
//               u chunk in registers), only the weights go through LDS.
#include "k_gemm.hpp"

namespace rmx {

// Output head for a last hidden layer too wide for one block: logit from the stored ReLU
// activations h[m][0..N) (one wave per row).
__global__ __launch_bounds__(256) void tower_head_kernel(int M, int N, const float* __restrict__ h, int ldh,
                                                         OutArgs oa) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float p = 0.f;
  for (int n = lane; n < N; n += 64) p += h[(int64_t)m * ldh + n] * oa.wo[n];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
  if (lane != 0) return;
  float y = p;
  if (oa.has_bo) y = y + oa.bo;
  if (oa.rowsum) {
    float rs = 0.f;
    for (int j = 0; j < oa.rowsum_k; ++j) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + j];
    y = rs + y;
  }
  if (oa.pre2) y = oa.pre2[m] + y;
  float t = oa.pre ? oa.pre[m] + y : y;
  t = t + oa.beta;
  oa.out[m] = 1.0f / (1.0f + expf(-t));
}

int launch_tower_head(hipStream_t s, int M, int N, const float* h, int ldh, const OutArgs& oa) {
  if (M <= 0) return RMX_OK;
  hipLaunchKernelGGL(tower_head_kernel, dim3((M + 3) / 4), dim3(256), 0, s, M, N, h, ldh, oa);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// C_l (H x F*Hp row-major, column f*Hp + h) -> [Hp_pad/16][F][Npad][16]
__global__ void pack_cin_kernel(const float* __restrict__ C, int F, int Hp, int H, int Npad, int64_t tot,
                                float* __restrict__ Wp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int kk = (int)(i & 15);
  const int64_t rest = i >> 4;
  const int n = (int)(rest % Npad);
  const int64_t c = rest / Npad;
  const int f = (int)(c % F);
  const int hc = (int)(c / F);
  const int h = hc * 16 + kk;
  Wp[i] = (n < H && h < Hp) ? C[(int64_t)n * F * Hp + (int64_t)f * Hp + h] : 0.f;
}

int launch_pack_cin(hipStream_t s, const float* mats, int F, CinLayer& L) {
  const int64_t tot = (int64_t)L.Hp_pad * F * L.Npad;
  hipLaunchKernelGGL(pack_cin_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats + L.w_off, F,
                     L.Hp, L.H, L.Npad, tot, L.W);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// The split CIN's K order (k_gemm.hpp cin_chunk).  Chunks run over h-chunks hc (16 maps each), and
// inside one over the fields f.  tri (layer 1, u = x0): z[f][h] = x0[f] x0[h] = z[h][f], so only
// h <= f is kept -- fields f >= 16 hc -- with C[f,h] + C[h,f] as the weight (CINEncoder.scala:152
// multiplies every ordered pair; the sum is the same bilinear form in one fp32 rounding per weight).
// pair: an h-chunk with <= 8 live maps (H = 200: maps 192..199) takes fields f0, f0 + 1 in one chunk
// (lane groups 0-1 and 2-3), so no MFMA runs on the zero half.
std::vector<int> cin_chunk_map(int F, int Hp, bool tri) {
  std::vector<int> m;
  const int nhc = (Hp + 15) / 16;
  for (int hc = 0; hc < nhc; ++hc) {
    const bool pair = Hp - 16 * hc <= 8;
    for (int f = tri ? 16 * hc : 0; f < F; f += pair ? 2 : 1) m.push_back(f | hc << 16 | (pair ? 1 << 30 : 0));
  }
  return m;
}

// C_l (H x F*Hp) -> [ncm][Npad][16] in the chunk-map order; element 4 g + q of chunk c is lane
// group g's K value q (plain: z[f0][16 hc + 4 g + q]; pair: z[f0 + g / 2][16 hc + 4 (g % 2) + q])
__global__ void pack_cin_map_kernel(const float* __restrict__ C, int F, int Hp, int H, int Npad, int tri,
                                    const int* __restrict__ cmap, int64_t tot, float* __restrict__ Wm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int e = (int)(i & 15), g = e >> 2, q = e & 3;
  const int64_t rest = i >> 4;
  const int n = (int)(rest % Npad);
  const int c = (int)(rest / Npad);
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

int launch_pack_cin_map(hipStream_t s, const float* mats, int F, CinLayer& L) {
  const int64_t tot = (int64_t)L.ncm * L.Npad * 16;
  if (tot <= 0) return RMX_OK;
  hipLaunchKernelGGL(pack_cin_map_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats + L.w_off, F,
                     L.Hp, L.H, L.Npad, L.tri, L.cmap, tot, L.Wm);
  RMX_HIP(hipGetLastError());
  return launch_pack_split3(s, L.Wm, L.ncm, L.Npad, L.W3);
}


// Npad of a tower layer of width N: a multiple of one block width NT*16 (NT from kNTs), chosen
// to minimise padding (ties: the wider block).
int tower_npad_for(int N) {
  const int nt = (N + 15) / 16;
  const bool even = tuning_get("tower_split", 1) != 0 && nt >= 8;  // tower variants 2/3 split NT in halves
  int best = -1, best_pad = 1 << 30;
  for (int c : kNTs) {
    if (even && c % 2) continue;
    const int pad = (nt + c - 1) / c * c;
    if (pad < best_pad || (pad == best_pad && c > best)) {
      best_pad = pad;
      best = c;
    }
  }
  return best_pad * 16;
}

// Npad of a CIN layer of H maps: one block spans the layer (the rowdot epilogue), so the
// smallest instantiated NT >= ceil(H/16); -1 if H is too wide.
int cin_npad_for(int H) {
  const int nt = (H + 15) / 16;
  for (int c : kCinNTs)
    if (c >= nt) return c * 16;
  return -1;
}

static int tower_nt_for(int Npad) {
  const int nt = Npad / 16;
  int best = 1;
  for (int c : kNTs)
    if (nt % c == 0 && c > best) best = c;
  return best;
}

static bool use_s3(const DenseLayer& L) { return L.W3 && f32_split_enabled() && L.Npad % kS3BN == 0; }

bool tower_wring(const DenseLayer& L, int M, const AGatherArgs* ga) {
  if (!ga || ga->k != 16 || M <= 0) return false;
  if (L.W16) {  // bf16: the 2-deep ring variants of launch_tower_nt (M >= 65,536, 26 tiles)
    if (M < 65536 || tower_nt_for(L.Npad) != 26) return false;
    const int var = tower_variant_for(26, Epi::kReluStore, true, L.K);
    return var == 4 || var == 5;
  }
  return use_s3(L) && tuning_get("s3_tower", 1) != 2;  // every split-GEMM tile but the register-staged one
}

bool tower_fm_fusable(const DenseLayer& L, int M, const AGatherArgs* ga, bool sums) {
  // every k = 16 gather kernel has the first-order epilogue; the FM sums need fp32 A fragments
  // (the split GEMM).  Knobs: fm_fuse (DeepFM first order + FM, default on: +4 % at the bench);
  // fo_fuse (the first order alone, xDeepFM / DCN): 0 off, 1 always, 2 (default) when layer 1
  // runs a w-ring tile (tower_wring: summed from LDS, free) -- the epilogue's own weight gathers
  // miss the caches (DCN bf16 -1 % at the bench)
  if (!ga || ga->k != 16 || ga->F > kFmMaxF) return false;
  if (sums) return tuning_get("fm_fuse", 1) != 0 && !L.W16 && use_s3(L);
  const int fo = tuning_get("fo_fuse", 2);
  return fo == 1 || (fo == 2 && tower_wring(L, M, ga));
}

int launch_tower_layer(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
                       const AGatherArgs* ga, float* C, int ldc, Epi epi, const OutArgs* oa, const XColArgs* xc,
                       const FmArgs* fm, bool cols32) {
  if (M <= 0) return RMX_OK;
  if (fm && (epi != Epi::kReluStore || !tower_fm_fusable(L, M, ga, fm->sums != 0))) {
    set_error("gemm: the fused first order + FM needs a gathered split-GEMM layer 1");
    return RMX_E_INVALID;
  }
  const int nt = tower_nt_for(L.Npad);
  if (epi == Epi::kOutput && nt * 16 != L.Npad) {
    // too wide for one block: store the ReLU activations, then a separate head pass
    if (L.W16) {
      set_error("bf16 tower: the last hidden layer must fit one block (N <= 416)");
      return RMX_E_INVALID;
    }
    int st = launch_tower_layer(s, L, M, A, lda, ga, C, ldc, Epi::kReluStore, nullptr, nullptr);
    if (st != RMX_OK) return st;
    hipLaunchKernelGGL(tower_head_kernel, dim3((M + 3) / 4), dim3(256), 0, s, M, L.N, C, ldc, *oa);
    RMX_HIP(hipGetLastError());
    return RMX_OK;
  }
  GemmArgs p{};
  p.M = M;
  p.K = L.K;
  p.Kpad = L.Kpad;
  p.Npad = L.Npad;
  p.A = A;
  p.lda = lda;
  if (ga) {
    p.ga = *ga;
    if (p.ga.ld == 0) p.ga.ld = p.ga.k;
    if (p.ga.ld < p.ga.k || (p.ga.k == 16 && (p.ga.ld & (p.ga.ld - 1)))) {
      set_error("gemm: table row stride must be >= k (a power of two at k = 16)");
      return RMX_E_INVALID;
    }
    p.gsh = __builtin_ctz((unsigned)p.ga.ld);
  }
  p.Wp = L.W16 ? reinterpret_cast<const float*>(L.W16) : L.W;
  p.bias = L.b;
  p.C = C;
  p.ldc = ldc;
  if (oa) p.oa = *oa;
  if (xc) {
    if (epi != Epi::kReluStore) {
      set_error("gemm: raw extra columns need the ReLU-store epilogue");
      return RMX_E_INVALID;
    }
    p.xcol = xc->ptr;
    p.xn_main = xc->n_main;
    p.xld = xc->ld;
  }
  if (fm) {
    p.fm_w = fm->w;
    p.fm_w_bf16 = fm->w_bf16;
    p.fm_sums = fm->sums;
    p.fm_add = fm->add;
    p.fm_y = fm->y;
    const int wld = fm->wld ? fm->wld : 1;
    if (wld & (wld - 1)) {
      set_error("gemm: first-order weight stride must be a power of two");
      return RMX_E_INVALID;
    }
    p.fm_wsh = __builtin_ctz((unsigned)wld);
  }
  const int amode = !ga ? kDenseA : (ga->k == 16 ? kGatherK16 : kGatherAny);
  if (L.W16) {
    const bool sliced = epi == Epi::kOutput && bf16_tower_sliced(L.Npad, epi, L.K, M, amode);
    if (sliced && !p.oa.part) {
      set_error("gemm: a sliced output layer needs the partial-logit buffer");
      return RMX_E_INVALID;
    }
    int st = launch_tower_bf16(s, p, nt, amode, epi);
    if (st == RMX_OK && sliced) st = launch_out_finish(s, M, L.Npad / kS3BN, *oa);
    return st;
  }
  if (use_s3(L) && (epi != Epi::kOutput || L.Npad == kS3BN || oa->part)) {
    // fp32 layer on the bf16 matrix cores through the exact 3-way split (k_gemm_s3.hip)
    p.Wp = reinterpret_cast<const float*>(L.W3);
    p.Kpad = (L.Kpad / 16 + 1) / 2 * 32;
    // cols32: DeepFM's column-split small-batch path (models.hip, knob "s3_cols") runs its dense-A layers on
    // 32-column blocks
    p.cols32 = cols32 && amode == kDenseA && L.Npad % 32 == 0 ? 1 : 0;
    const int bn = p.cols32 ? 32 : kS3BN;
    int st = launch_tower_s3(s, p, amode, epi);
    if (st == RMX_OK && epi == Epi::kOutput && L.Npad > bn) st = launch_out_finish(s, M, L.Npad / bn, *oa);
    return st;
  }
  switch (nt) {
#define RMX_NT(n) \
  case n: return launch_tower_nt<n, kPrecF32>(s, p, amode, epi);
    RMX_NT(1) RMX_NT(2) RMX_NT(3) RMX_NT(4) RMX_NT(5) RMX_NT(6) RMX_NT(7)
    RMX_NT(8) RMX_NT(10) RMX_NT(13) RMX_NT(16) RMX_NT(20) RMX_NT(25) RMX_NT(26)
#undef RMX_NT
    default: set_error("bad tower width"); return RMX_E_INVALID;
  }
}

int launch_cin_layer(hipStream_t s, const CinLayer& L, bool first, bool last, int B, int F, int k,
                     const int32_t* ids, const float* table, const float* u_prev, float* u_out, float* rowdot,
                     int ld) {
  if (B <= 0) return RMX_OK;
  if (!first && !u_prev) {
    set_error("cin: missing previous layer maps");
    return RMX_E_INVALID;
  }
  GemmArgs p{};
  p.M = B * k;
  p.K = L.Hp_pad * F;
  p.Kpad = p.K;
  p.Npad = L.Npad;
  p.ga = AGatherArgs{ids, table, F, k, ld > 0 ? ld : k};
  p.u_prev = u_prev;
  p.ldu = L.Hp_pad;
  p.XS = round_up(std::max(F, first ? L.Hp_pad : 0), 16) + 4;  // 16-B rows; x0 and (layer 1) u
  p.cin_first = first ? 1 : 0;
  p.Wp = L.W;
  p.bias = L.b;
  p.C = last ? nullptr : u_out;
  p.ldc = L.Npad;
  p.wo = L.wo;
  p.rowdot = rowdot;
  if (p.K / 16 + 8 >= 65536 || F >= 65536) {  // the kernel's exact c16 / F (k_gemm.hpp div_f)
    set_error("cin: F * H_prev must stay below 1,048,448");
    return RMX_E_INVALID;
  }
  if (first && L.Hp_pad > p.XS - 4) {
    set_error("cin: first layer Hp_pad mismatch");
    return RMX_E_INVALID;
  }
  if (L.W3 && f32_split_enabled() && L.Npad == kS3BN) {
    p.Wp = reinterpret_cast<const float*>(L.W3);
    p.cin_pair_hc = -1;
    if (L.map_on) {  // W3 packed in the chunk-map order (cin_chunk_map)
      p.K = L.ncm * 16;
      if (L.tri || tuning_get("cin_map_lds", 0)) {  // the triangle: entries staged in LDS
        p.cmap = L.cmap;
        p.ncmap = L.ncm;
      } else {  // decoded in closed form (k_gemm.hpp cin_chunk)
        const int last = (L.Hp + 15) / 16 - 1;
        if (L.Hp - 16 * last <= 8) p.cin_pair_hc = last;
      }
    }
    p.Kpad = round_up(p.K, 32);
    return launch_cin_s3(s, p);
  }
  switch (L.Npad / 16) {
#define RMX_NT(n) \
  case n: return launch_cin_nt<n>(s, p);
    RMX_NT(1) RMX_NT(2) RMX_NT(3) RMX_NT(4) RMX_NT(5) RMX_NT(6) RMX_NT(7)
    RMX_NT(8) RMX_NT(10) RMX_NT(13) RMX_NT(16)
#undef RMX_NT
    default:
      set_error("cin: layer width must be <= 256");
      return RMX_E_INVALID;
  }
}

}  // namespace rmx
