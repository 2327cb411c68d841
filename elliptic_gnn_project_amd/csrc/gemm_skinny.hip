// K7s — skinny GEMM shapes of the convs' narrow output layers, on the vector ALUs.
//
// GCN / GAT / SAGE-ResBN end in a Linear with out_channels = num_classes = 2
// (src/models/gnn.py:23, :66, :124), so three of their GEMMs are [2e5, 64] x [64, 2],
// its transpose-product dW = Gᵀ·A with G [2e5, 2], and the input gradient [2e5, 2] x [2, 64].
// A 128-column MFMA tile wastes > 95 % of its work on them and still pays the tile machinery;
// these are pure HBM streams (one read of A or one write of C), so they run as wave-level
// FMA kernels at full f32 accuracy (either gnn_gemm_math mode):
//   nt_skinny_n  C[M, Nc <= 8]  = A[M, K <= 384] · Wᵀ   — lane groups split K, xor-shuffle reduce
//   nt_skinny_k  C[M, Nc]       = A[M, K <= 8] · B      — B in registers, one VEC-column slot per lane
//   tn_skinny    dW[Nr <= 8, K] = Gᵀ·A and db = Σ G     — per-block partials into the TN slab
// Epilogue semantics (bias, ReLU, counter-hash dropout) are the NT kernels' (gemm_common.hpp).
#include <algorithm>

#include "gemm_common.hpp"

namespace gnnmp {
namespace {

template <int VEC>
struct Vf { float v[VEC]; };

template <int VEC>
__device__ __forceinline__ Vf<VEC> ldf(const float* p) {
  Vf<VEC> r;
  if constexpr (VEC == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (VEC == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = *p;
  }
  return r;
}

__device__ __forceinline__ uint64_t nt_seed(const NTArgs& a) {
  return a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
}

__device__ __forceinline__ float nt_epi(const NTArgs& a, float v, int64_t row, int col, uint64_t seed) {
  if (a.bias) v += a.bias[col];
  if (a.relu) v = fmaxf(v, 0.0f);
  if (a.dropout)
    v = keep_elem(seed, (uint32_t)row * (uint32_t)a.Nc + (uint32_t)col, a.keep_thresh) ? v * a.drop_scale : 0.0f;
  if (a.mask) v = a.mask[row * a.ldmask + col] > 0.0f ? v * a.mask_scale : 0.0f;
  return v;
}

constexpr int SK_MAXN = 8;
constexpr int kSkU = 4;  // rows in flight per thread in the skinny NT kernels
constexpr int SK_KMAX = KMAX;  // 384

// C[r, n] = Σ_k A[r, k] W[n, k]: TPR lanes per row each own K/VEC/TPR chunks of VEC columns,
// W staged once per block in LDS ([n][k]), the Nc partial dots reduced over the row's lanes.
template <int VEC, int NC>
__global__ __launch_bounds__(256) void nt_skinny_n_kernel(NTArgs a, int lg_tpr) {
  __shared__ float ws[SK_MAXN * SK_KMAX];
  const int K = a.k1 + a.k2;
  for (int i = threadIdx.x; i < NC * K; i += 256) {  // rows Nc..NC-1 zero (their dots are discarded)
    const int n = i / K, k = i - n * K;
    float w;
    if (n >= a.Nc) w = 0.0f;
    else if (a.bt) w = a.bt[(int64_t)k * a.ldb + n];
    else w = k < a.k1 ? a.w1[(int64_t)n * a.ldw1 + k] : a.w2[(int64_t)n * a.ldw2 + (k - a.k1)];
    ws[i] = w;
  }
  __syncthreads();
  const int TPR = 1 << lg_tpr;
  const int lig = threadIdx.x & (TPR - 1);
  const int rpb = 256 >> lg_tpr;
  const int nch = K / VEC;
  const uint64_t seed = a.dropout ? nt_seed(a) : 0;
  // kSkU rows per thread per pass (block-uniform trip count: every lane reaches the shuffles), the
  // rows' A chunks loaded together from clamped rows
  const int64_t stride = (int64_t)gridDim.x * rpb;
  for (int64_t b0 = (int64_t)blockIdx.x * rpb; b0 < a.M; b0 += kSkU * stride) {
    const int64_t rt = b0 + (threadIdx.x >> lg_tpr);
    float acc[kSkU][NC];
#pragma unroll
    for (int u = 0; u < kSkU; ++u)
#pragma unroll
      for (int n = 0; n < NC; ++n) acc[u][n] = 0.0f;
    for (int c = lig; c < nch; c += TPR) {
      const int k = c * VEC;
      Vf<VEC> x[kSkU];
#pragma unroll
      for (int u = 0; u < kSkU; ++u) {
        const int64_t r = rt + u * stride < a.M ? rt + u * stride : (rt < a.M ? rt : b0);
        x[u] = ldf<VEC>(k < a.k1 ? a.a1 + r * a.lda1 + k : a.a2 + r * a.lda2 + (k - a.k1));
      }
#pragma unroll
      for (int u = 0; u < kSkU; ++u)
#pragma unroll
        for (int n = 0; n < NC; ++n)
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[u][n] = fmaf(x[u].v[i], ws[n * K + k + i], acc[u][n]);
    }
#pragma unroll
    for (int u = 0; u < kSkU; ++u)
      for (int off = TPR >> 1; off >= 1; off >>= 1) {
#pragma unroll
        for (int n = 0; n < NC; ++n) acc[u][n] += __shfl_xor(acc[u][n], off);
      }
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      const int64_t r = rt + u * stride;
      if (r < a.M && lig < a.Nc) {
        float v = acc[u][0];
#pragma unroll
        for (int n = 1; n < NC; ++n) v = lig == n ? acc[u][n] : v;
        v = nt_epi(a, v, r, lig, seed);
        if (a.c) a.c[r * a.ldc + lig] = v;
      }
    }
  }
}

// C[r, n0..n0+VEC) = Σ_{k<K} A[r, k] B[k, n0..]: B's K x VEC slice of a lane in registers,
// the row's K values broadcast to its TPR lanes.
// colsum_part (optional): block b's column sums of the C it stores, colsum_part[b·Nc + n] — each
// thread sums its rows in order, the block's row groups are added in order through LDS (the bias
// gradient of the layer whose masked input gradient this is: no separate pass over C)
template <int VEC, int KK>
__global__ __launch_bounds__(256) void nt_skinny_k_kernel(NTArgs a, int lg_tpr) {
  __shared__ float csl[256 * VEC];
  const int TPR = 1 << lg_tpr;
  const int lig = threadIdx.x & (TPR - 1);
  const int rpb = 256 >> lg_tpr;
  const int n0 = lig * VEC;
  const bool col_ok = n0 < a.Nc;
  float b[KK][VEC];
#pragma unroll
  for (int k = 0; k < KK; ++k)
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float w = 0.0f;
      if (col_ok && k < a.k1)
        w = a.bt ? a.bt[(int64_t)k * a.ldb + n0 + i] : a.w1[(int64_t)(n0 + i) * a.ldw1 + k];
      b[k][i] = w;
    }
  const uint64_t seed = a.dropout ? nt_seed(a) : 0;
  float cs[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) cs[i] = 0.0f;
  // kSkU rows per thread per pass, their A values loaded together (clamped rows) before any store
  // (one row per pass left one dependent load → store round trip per row: 35 us for [203769, 64])
  const int64_t stride = (int64_t)gridDim.x * rpb;
  for (int64_t r0 = (int64_t)blockIdx.x * rpb + (threadIdx.x >> lg_tpr); col_ok && r0 < a.M; r0 += kSkU * stride) {
    float av[kSkU][KK];
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      const int64_t r = r0 + u * stride < a.M ? r0 + u * stride : r0;
#pragma unroll
      for (int k = 0; k < KK; ++k) av[u][k] = a.a1[r * a.lda1 + (k < a.k1 ? k : 0)];
    }
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      const int64_t r = r0 + u * stride;
      if (r >= a.M) break;
      float o[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float s = av[u][0] * b[0][i];
#pragma unroll
        for (int k = 1; k < KK; ++k) s = fmaf(k < a.k1 ? av[u][k] : 0.0f, b[k][i], s);
        o[i] = nt_epi(a, s, r, n0 + i, seed);
        cs[i] += o[i];
      }
      if (!a.c) continue;
      float* dst = a.c + r * a.ldc + n0;
      if constexpr (VEC == 4) *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
      else if constexpr (VEC == 2) *reinterpret_cast<float2*>(dst) = make_float2(o[0], o[1]);
      else *dst = o[0];
    }
  }
  if (!a.colsum_part) return;  // kernel-uniform
#pragma unroll
  for (int i = 0; i < VEC; ++i) csl[i * 256 + threadIdx.x] = cs[i];
  __syncthreads();
  if ((threadIdx.x >> lg_tpr) == 0 && col_ok) {  // row group 0: the rpb groups' sums in order
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float t = csl[i * 256 + lig];
      for (int g = 1; g < rpb; ++g) t += csl[i * 256 + g * TPR + lig];
      if (n0 + i < a.Nc) a.colsum_part[(int64_t)blockIdx.x * a.Nc + n0 + i] = t;
    }
  }
}

// Block b: dW partial over its rows [b·rpb, (b+1)·rpb) into slab[b] (dW1 [Nr, k1] | dW2 [Nr, k2]), db into
// slab[b][Nr·K + n].  Row groups reduce through LDS in fixed order (deterministic).
template <int VEC, int NR>
__global__ __launch_bounds__(256) void tn_skinny_kernel(TNArgs a, int lg_tpr) {
  __shared__ float red[256 * NR * VEC];
  __shared__ float redb[256 * NR];
  const int K = a.k1 + a.k2;
  const int TPR = 1 << lg_tpr;
  const int RG = 256 >> lg_tpr;
  const int lig = threadIdx.x & (TPR - 1);
  const int rg = threadIdx.x >> lg_tpr;
  const int nch = K / VEC;
  const bool ch_ok = lig < nch;
  const int k = lig * VEC;
  const int64_t rb = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t re = rb + a.rows_per_block < a.M ? rb + a.rows_per_block : a.M;
  float acc[NR][VEC], gs[NR];
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    gs[n] = 0.0f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[n][i] = 0.0f;
  }
  const float* abase = k < a.k1 ? a.a1 + k : a.a2 + (k - a.k1);
  const int64_t lda = k < a.k1 ? a.lda1 : a.lda2;
#pragma unroll 4
  for (int64_t r = rb + rg; r < re; r += RG) {
    float g[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) g[n] = n < a.Nr ? a.g[r * a.ldg + n] : 0.0f;
    if (ch_ok) {
      const Vf<VEC> x = ldf<VEC>(abase + r * lda);
#pragma unroll
      for (int n = 0; n < NR; ++n)
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[n][i] = fmaf(g[n], x.v[i], acc[n][i]);
    }
#pragma unroll
    for (int n = 0; n < NR; ++n) gs[n] += g[n];
  }
  // red[rg][n][k + i]  (K <= TPR·VEC, so the image is RG x NR x TPR·VEC <= 256·NR·VEC floats)
  const int W = TPR * VEC;
#pragma unroll
  for (int n = 0; n < NR; ++n)
#pragma unroll
    for (int i = 0; i < VEC; ++i) red[(rg * NR + n) * W + k + i] = acc[n][i];
  if (lig == 0) {
#pragma unroll
    for (int n = 0; n < NR; ++n) redb[rg * NR + n] = gs[n];
  }
  __syncthreads();
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  for (int o = threadIdx.x; o < a.Nr * K; o += 256) {
    const int n = o / K, kk = o - n * K;
    float s = 0.0f;
    for (int q = 0; q < RG; ++q) s += red[(q * NR + n) * W + kk];
    // TN output layout is segment-major: dW1 [Nr, k1], then dW2 [Nr, k2]
    slab[kk < a.k1 ? n * a.k1 + kk : a.Nr * a.k1 + n * a.k2 + (kk - a.k1)] = s;
  }
  if (threadIdx.x < a.Nr) {
    float s = 0.0f;
    for (int q = 0; q < RG; ++q) s += redb[q * NR + threadIdx.x];
    slab[a.Nr * K + threadIdx.x] = s;
  }
}

int lg2ceil(int v) { int l = 0; while ((1 << l) < v) ++l; return l; }
bool al(const void* p, int b) { return (reinterpret_cast<uintptr_t>(p) % (uintptr_t)b) == 0; }

unsigned grid_for(int64_t M, int rpb, int64_t cap) {
  int64_t b = ceil_div(M, rpb);
  if (b > cap) b = cap;
  return (unsigned)(b > 0 ? b : 1);
}

}  // namespace

// the skinny-K form's VEC and grid (launch_nt_skinny below); 0 blocks: not that form
static int skk_vec(const NTArgs& a) {
  auto c_ok = [&](int v) { return a.Nc % v == 0 && (!a.c || (a.ldc % v == 0 && al(a.c, 4 * v))); };
  return c_ok(4) ? 4 : (c_ok(2) ? 2 : 1);
}
int nt_skinny_k_blocks(const NTArgs& a) {
  if (a.a_bf16 || a.c_bf16 || a.nproj > 0 || a.M == 0 || a.Nc <= SK_MAXN) return 0;
  if (!(a.k2 == 0 && a.k1 <= SK_MAXN && a.Nc <= 64 * 4)) return 0;
  const int lg = lg2ceil((a.Nc + skk_vec(a) - 1) / skk_vec(a));
  if (lg > 8) return 0;
  return (int)grid_for(ceil_div(a.M, kSkU), 256 >> lg, 8192);
}

bool launch_nt_skinny(const NTArgs& a, hipStream_t st) {
  if (a.a_bf16 || a.c_bf16 || a.nproj > 0 || a.M == 0) return false;
  const int K = a.k1 + a.k2;
  if (a.Nc <= SK_MAXN && K <= SK_KMAX) {
    if (a.colsum_part) return false;  // (the column sums ride only in the skinny-K form)
    auto v_ok = [&](int v) {
      return a.k1 % v == 0 && a.lda1 % v == 0 && al(a.a1, 4 * v) &&
             (a.k2 == 0 || (a.k2 % v == 0 && a.lda2 % v == 0 && al(a.a2, 4 * v)));
    };
    const int VEC = v_ok(4) ? 4 : (v_ok(2) ? 2 : 1);
    // TPR lanes per row: enough for K/VEC chunks (capped at a wave) and at least Nc, since lane
    // n of the row writes column n
    const int lg = std::max(lg2ceil(a.Nc), std::min(6, lg2ceil(K / VEC)));
    const unsigned nb = grid_for(ceil_div(a.M, kSkU), 256 >> lg, 8192);
    const int NC = a.Nc <= 1 ? 1 : a.Nc <= 2 ? 2 : a.Nc <= 4 ? 4 : 8;
#define GNN_SKN(V, N) nt_skinny_n_kernel<V, N><<<nb, 256, 0, st>>>(a, lg)
#define GNN_SKN_V(V) \
  if (NC == 1) GNN_SKN(V, 1); else if (NC == 2) GNN_SKN(V, 2); else if (NC == 4) GNN_SKN(V, 4); else GNN_SKN(V, 8)
    if (VEC == 4) { GNN_SKN_V(4); } else if (VEC == 2) { GNN_SKN_V(2); } else { GNN_SKN_V(1); }
#undef GNN_SKN_V
#undef GNN_SKN
    return true;
  }
  if (a.k2 == 0 && a.k1 <= SK_MAXN && a.Nc <= 64 * 4) {
    const int VEC = skk_vec(a);
    const int lg = lg2ceil((a.Nc + VEC - 1) / VEC);
    if (lg > 8) return false;
    const unsigned nb = grid_for(ceil_div(a.M, kSkU), 256 >> lg, 8192);
    const int KK = a.k1 <= 1 ? 1 : a.k1 <= 2 ? 2 : a.k1 <= 4 ? 4 : 8;
#define GNN_SKK(V, KX) nt_skinny_k_kernel<V, KX><<<nb, 256, 0, st>>>(a, lg)
#define GNN_SKK_V(V) \
  if (KK == 1) GNN_SKK(V, 1); else if (KK == 2) GNN_SKK(V, 2); else if (KK == 4) GNN_SKK(V, 4); else GNN_SKK(V, 8)
    if (VEC == 4) { GNN_SKK_V(4); } else if (VEC == 2) { GNN_SKK_V(2); } else { GNN_SKK_V(1); }
#undef GNN_SKK_V
#undef GNN_SKK
    return true;
  }
  return false;
}

int tn_skinny_blocks(int64_t M) {
  int64_t b = ceil_div(M, 256);
  if (b > 1024) b = 1024;
  return (int)(b > 0 ? b : 1);
}

int tn_vec(const TNArgs& a);

bool tn_skinny_ok(const TNArgs& a) {
  return a.Nr <= SK_MAXN && !a.dz && !a.h && !a.gout && !a.a_bf16 && a.g && a.k1 + a.k2 <= SK_KMAX &&
         lg2ceil((a.k1 + a.k2) / tn_vec(a)) <= 8;
}

int tn_vec(const TNArgs& a) {
  auto v_ok = [&](int v) {
    return a.k1 % v == 0 && a.lda1 % v == 0 && al(a.a1, 4 * v) &&
           (a.k2 == 0 || (a.k2 % v == 0 && a.lda2 % v == 0 && al(a.a2, 4 * v)));
  };
  return v_ok(4) ? 4 : (v_ok(2) ? 2 : 1);
}

void launch_tn_skinny(const TNArgs& a0, int nblk, hipStream_t st) {
  TNArgs a = a0;
  a.rows_per_block = ceil_div(a.M, nblk);
  const int K = a.k1 + a.k2;
  const int VEC = tn_vec(a);
  const int lg = lg2ceil(K / VEC);  // all K/VEC chunks of a row at once (<= 256 lanes, tn_skinny_ok)
  const int NR = a.Nr <= 1 ? 1 : a.Nr <= 2 ? 2 : a.Nr <= 4 ? 4 : 8;
#define GNN_SKT(V, N) tn_skinny_kernel<V, N><<<nblk, 256, 0, st>>>(a, lg)
#define GNN_SKT_V(V) \
  if (NR == 1) GNN_SKT(V, 1); else if (NR == 2) GNN_SKT(V, 2); else if (NR == 4) GNN_SKT(V, 4); else GNN_SKT(V, 8)
  if (VEC == 4) { GNN_SKT_V(4); } else if (VEC == 2) { GNN_SKT_V(2); } else { GNN_SKT_V(1); }
#undef GNN_SKT_V
#undef GNN_SKT
}

}  // namespace gnnmp
