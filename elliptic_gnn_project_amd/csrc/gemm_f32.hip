// K7 — fp32 MFMA GEMMs for the dense transforms of SAGEConv/GCNConv/GATConv, with the
// surrounding elementwise work of src/models/gnn.py fused in.
//
// Replaces PyG Linear (lin_l / lin_r / lin, gnn.py:41-44, 20-23, 64-67) and the ReLU +
// dropout between layers (gnn.py:29-30, 50-51) — forward (NT kernel) and weight
// gradients (TN kernel).  Exact fp32: v_mfma_f32_32x32x2_f32 is a k-ordered fmaf chain
// (no TF32/xf32 on gfx950), so results are within fp32 rounding of ATen's sgemm.
//
// NT:  C[M,Nc] = epi( [A1 | A2][M, k1+k2] · Bt[k1+k2, Nc] )
//      epi = +bias, ReLU, dropout (counter hash, keep prob 1-p, scale 1/(1-p)),
//      optional projection Z[M,nproj] = C · Pᵀ (P [nproj, Nc]) — the next, narrow layer's
//      transform-first GEMM computed from registers (the hidden activations' row is whole
//      in one wave).  Block = 4 waves x (32 rows x 128 cols); K streamed in 32-deep chunks
//      through double-buffered LDS (A padded to 33 floats/row: conflict-free b32 reads).
// TN:  dW[Nr, k1+k2] = Σ_m G[m, Nr]ᵀ · [A1 | A2][m, :]   (split over M, slabs, ordered reduce)
//      G = (G_src or dz·P) ⊙ (h > 0 ? scale : 0)   — ReLU+dropout backward computed on the fly
//      side sums: db[n] = Σ G, dW2[q][n] = Σ dz[m,q]·h[m,n], dzsum[q] = Σ dz[m,q]
//      Block = 8 waves: wave w owns dW rows (w&3)*32.. and k-tiles (w>>2)*6 .. +6.
// Both are atomic-free and deterministic.
#include "common.hpp"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace gnnmp {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Dropout keep decision for element `idx` of a call seeded with `seed` (mirrored bit for
// bit by oracle/dropout_hash.py so CPU parity can use the same masks).
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, uint32_t keep_thresh) {
  return (uint32_t)(mix64(seed ^ (idx * 0xD1B54A32D192ED03ull)) >> 40) < keep_thresh;
}

namespace {

constexpr int BM = 128, BN = 128, KC = 32, APITCH = KC + 1;

struct NTArgs {
  int64_t M;
  int32_t Nc;
  const float* a1; int64_t lda1; int32_t k1;
  const float* a2; int64_t lda2; int32_t k2;
  const float* bt; int64_t ldb;
  float* c; int64_t ldc;
  const float* bias;
  int32_t relu;
  int32_t dropout; uint32_t keep_thresh; float drop_scale; uint64_t seed;
  const float* proj; int32_t nproj; float* z; int64_t ldz;
};

template <int AVEC>
__device__ __forceinline__ void nt_load_a(const NTArgs& a, int c, int64_t m0, float (&ra)[16]) {
  const int nch1 = (a.k1 + KC - 1) / KC;
  const float* A; int64_t lda; int k0, klen;
  if (c < nch1) { A = a.a1; lda = a.lda1; k0 = c * KC; klen = min(KC, a.k1 - k0); }
  else { A = a.a2; lda = a.lda2; k0 = (c - nch1) * KC; klen = min(KC, a.k2 - k0); }
  constexpr int VPR = KC / AVEC;  // vectors per row
#pragma unroll
  for (int i = 0; i < 16 / AVEC; ++i) {
    int v = threadIdx.x + 256 * i;
    int r = v / VPR;
    int k = (v % VPR) * AVEC;
    int64_t row = m0 + r;
    const float* p = A + row * lda + k0 + k;
    if (row < a.M && k + AVEC <= klen) {
      if constexpr (AVEC == 4) {
        float4 t = *reinterpret_cast<const float4*>(p);
        ra[i * 4 + 0] = t.x; ra[i * 4 + 1] = t.y; ra[i * 4 + 2] = t.z; ra[i * 4 + 3] = t.w;
      } else if constexpr (AVEC == 2) {
        float2 t = *reinterpret_cast<const float2*>(p);
        ra[i * 2 + 0] = t.x; ra[i * 2 + 1] = t.y;
      } else {
        ra[i] = *p;
      }
    } else {
#pragma unroll
      for (int q = 0; q < AVEC; ++q) ra[i * AVEC + q] = (row < a.M && k + q < klen) ? p[q] : 0.0f;
    }
  }
}

template <int AVEC>
__device__ __forceinline__ void nt_store_a(float* As, const float (&ra)[16]) {
  constexpr int VPR = KC / AVEC;
#pragma unroll
  for (int i = 0; i < 16 / AVEC; ++i) {
    int v = threadIdx.x + 256 * i;
    int r = v / VPR;
    int k = (v % VPR) * AVEC;
#pragma unroll
    for (int q = 0; q < AVEC; ++q) As[r * APITCH + k + q] = ra[i * AVEC + q];
  }
}

__device__ __forceinline__ void nt_load_b(const NTArgs& a, int c, int n0, bool vec4, float (&rb)[16]) {
  const int nch1 = (a.k1 + KC - 1) / KC;
  int kb0, klen;
  if (c < nch1) { kb0 = c * KC; klen = min(KC, a.k1 - c * KC); }
  else { int cc = c - nch1; kb0 = a.k1 + cc * KC; klen = min(KC, a.k2 - cc * KC); }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int v = threadIdx.x + 256 * i;  // 1024 float4 slots = 32 rows x 32
    int kk = v >> 5;
    int n = (v & 31) * 4;
    const float* p = a.bt + (int64_t)(kb0 + kk) * a.ldb + n0 + n;
    if (vec4 && kk < klen && n0 + n + 4 <= a.Nc) {
      float4 t = *reinterpret_cast<const float4*>(p);
      rb[i * 4 + 0] = t.x; rb[i * 4 + 1] = t.y; rb[i * 4 + 2] = t.z; rb[i * 4 + 3] = t.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) rb[i * 4 + q] = (kk < klen && n0 + n + q < a.Nc) ? p[q] : 0.0f;
    }
  }
}

__device__ __forceinline__ void nt_store_b(float* Bs, const float (&rb)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int v = threadIdx.x + 256 * i;
    int kk = v >> 5;
    int n = (v & 31) * 4;
    *reinterpret_cast<float4*>(&Bs[kk * BN + n]) = make_float4(rb[i * 4], rb[i * 4 + 1], rb[i * 4 + 2], rb[i * 4 + 3]);
  }
}

__device__ __forceinline__ int chunk_ksteps(const NTArgs& a, int c) {
  const int nch1 = (a.k1 + KC - 1) / KC;
  int klen = (c < nch1) ? min(KC, a.k1 - c * KC) : min(KC, a.k2 - (c - nch1) * KC);
  return (klen + 1) >> 1;
}

template <int AVEC>
__global__ __launch_bounds__(256) void gemm_nt_kernel(NTArgs a) {
  __shared__ float As[2][BM * APITCH];
  __shared__ __attribute__((aligned(16))) float Bs[2][KC * BN];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nchunks = (a.k1 + KC - 1) / KC + (a.k2 + KC - 1) / KC;
  const bool bvec4 = ((a.ldb & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.bt) & 15) == 0);

  floatx16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  float ra[16], rb[16];
  nt_load_a<AVEC>(a, 0, m0, ra);
  nt_load_b(a, 0, n0, bvec4, rb);
  nt_store_a<AVEC>(As[0], ra);
  nt_store_b(Bs[0], rb);
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunks) {
      nt_load_a<AVEC>(a, c + 1, m0, ra);
      nt_load_b(a, c + 1, n0, bvec4, rb);
    }
    const float* Aw = As[buf] + (wave * 32 + (lane & 31)) * APITCH + (lane >> 5);
    const float* Bw = Bs[buf] + (lane >> 5) * BN + (lane & 31);
    const int ks = chunk_ksteps(a, c);
    for (int s = 0; s < ks; ++s) {
      const float af = Aw[2 * s];
      const float* b = Bw + 2 * s * BN;
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, b[t * 32], acc[t], 0, 0, 0);
    }
    if (c + 1 < nchunks) {
      nt_store_a<AVEC>(As[buf ^ 1], ra);
      nt_store_b(Bs[buf ^ 1], rb);
    }
    __syncthreads();
  }

  // ---------------- epilogue: bias, ReLU, dropout, store, optional projection
  const int64_t rbase = m0 + wave * 32 + 4 * (lane >> 5);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int col = n0 + t * 32 + (lane & 31);
    const bool colok = col < a.Nc;
    const float bv = (a.bias && colok) ? a.bias[col] : 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
      float v = acc[t][r] + bv;
      if (a.relu) v = fmaxf(v, 0.0f);
      if (a.dropout) v = keep_elem(a.seed, (uint64_t)row * (uint64_t)a.Nc + (uint64_t)col, a.keep_thresh) ? v * a.drop_scale : 0.0f;
      if (!colok) v = 0.0f;
      if (a.c && row < a.M && colok) a.c[row * a.ldc + col] = v;
      acc[t][r] = v;
    }
  }
  if (a.nproj > 0) {
    for (int q = 0; q < a.nproj; ++q) {
      float pw[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = n0 + t * 32 + (lane & 31);
        pw[t] = col < a.Nc ? a.proj[(int64_t)q * a.Nc + col] : 0.0f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float s = acc[0][r] * pw[0];
        s = fmaf(acc[1][r], pw[1], s);
        s = fmaf(acc[2][r], pw[2], s);
        s = fmaf(acc[3][r], pw[3], s);
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) s += __shfl_xor(s, off);
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
        if ((lane & 31) == 0 && row < a.M) a.z[row * a.ldz + q] = s;
      }
    }
  }
}

// ------------------------------------------------------------------------------------ TN
constexpr int MC = 32;          // rows per chunk
constexpr int TN_WAVES = 8;
constexpr int KT_PER_WAVE = 6;  // k-tiles per wave -> Kc <= 2 * 6 * 32 = 384
constexpr int KMAX = 2 * KT_PER_WAVE * 32;
constexpr int TN_APITCH = KMAX;
constexpr int MAXPROJ = 4;

struct TNArgs {
  int64_t M;
  int32_t Nr;
  const float* g; int64_t ldg;
  const float* dz; int64_t lddz; const float* proj; int32_t nproj;
  const float* h; int64_t ldh; float hscale;
  float* gout; int64_t ldgout;
  const float* a1; int64_t lda1; int32_t k1;
  const float* a2; int64_t lda2; int32_t k2;
  float* slab; int64_t slab_stride;
  int64_t rows_per_block;
  int32_t want_db;
};

// slab layout: dW[Nr][Kc] | db[Nr] | dW2[nproj][Nr] | dzsum[nproj]
__global__ __launch_bounds__(512) void gemm_tn_kernel(TNArgs a) {
  __shared__ __attribute__((aligned(16))) float Gs[MC * 128];
  __shared__ __attribute__((aligned(16))) float As[MC * TN_APITCH];
  __shared__ float red[4 * 128 * (1 + MAXPROJ)];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ntile = wave & 3;
  const int kt0 = (wave >> 2) * KT_PER_WAVE;
  const int Kc = a.k1 + a.k2;
  const int nkt = (Kc + 31) / 32;
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);

  floatx16 acc[KT_PER_WAVE];
#pragma unroll
  for (int t = 0; t < KT_PER_WAVE; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  // prologue thread mapping: column n = tid & 127, rows rg*8 .. rg*8+7
  const int pn = tid & 127;
  const int rg = tid >> 7;
  float db = 0.0f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float dzs[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float pcol[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  if (a.dz) {
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) pcol[q] = (q < a.nproj && pn < a.Nr) ? a.proj[q * a.Nr + pn] : 0.0f;
  }

  for (int64_t m0 = mbeg; m0 < mend; m0 += MC) {
    // ---- G chunk (prologue: recompute ReLU/dropout backward, side sums)
#pragma unroll
    for (int i = 0; i < MC / 4; ++i) {
      const int r = rg * (MC / 4) + i;
      const int64_t m = m0 + r;
      float g = 0.0f;
      if (m < mend && pn < a.Nr) {
        float dzv[MAXPROJ];
        if (a.dz) {
#pragma unroll
          for (int q = 0; q < MAXPROJ; ++q) dzv[q] = q < a.nproj ? a.dz[m * a.lddz + q] : 0.0f;
          g = dzv[0] * pcol[0];
#pragma unroll
          for (int q = 1; q < MAXPROJ; ++q) g = fmaf(dzv[q], pcol[q], g);
        } else {
          g = a.g[m * a.ldg + pn];
        }
        if (a.h) {
          const float hv = a.h[m * a.ldh + pn];
          g = hv > 0.0f ? g * a.hscale : 0.0f;
          if (a.dz) {
#pragma unroll
            for (int q = 0; q < MAXPROJ; ++q) dw2[q] = fmaf(dzv[q], hv, dw2[q]);
          }
        }
        if (a.dz && pn == 0) {
#pragma unroll
          for (int q = 0; q < MAXPROJ; ++q) dzs[q] += dzv[q];
        }
        db += g;
        if (a.gout) a.gout[m * a.ldgout + pn] = g;
      }
      Gs[r * 128 + pn] = g;
    }
    // ---- A chunk: rows m0.., columns [0, Kc) of [A1 | A2], zero padded to nkt*32
    const int kpad = nkt * 32;
    for (int v = tid; v < MC * kpad; v += 512) {
      const int r = v / kpad;
      const int k = v - r * kpad;
      const int64_t m = m0 + r;
      float x = 0.0f;
      if (m < mend) {
        if (k < a.k1) x = a.a1[m * a.lda1 + k];
        else if (k < Kc) x = a.a2[m * a.lda2 + (k - a.k1)];
      }
      As[r * TN_APITCH + k] = x;
    }
    __syncthreads();
    // ---- MFMA: dW[ntile rows][k tiles] += Gᵀ · A over these MC rows
    const float* gptr = Gs + (lane >> 5) * 128 + ntile * 32 + (lane & 31);
    const float* aptr = As + (lane >> 5) * TN_APITCH + (lane & 31);
    for (int s = 0; s < MC / 2; ++s) {
      const float gf = gptr[2 * s * 128];
#pragma unroll
      for (int t = 0; t < KT_PER_WAVE; ++t) {
        if (kt0 + t < nkt) {
          const float af = aptr[2 * s * TN_APITCH + (kt0 + t) * 32];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(gf, af, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  // ---- write this block's partial dW
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int t = 0; t < KT_PER_WAVE; ++t) {
    const int kt = kt0 + t;
    if (kt >= nkt) continue;
    const int col = kt * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = ntile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < a.Nr && col < Kc) slab[(int64_t)row * Kc + col] = acc[t][r];
    }
  }
  // ---- side sums: reduce the 4 row groups through LDS (fixed order)
  const int ns = 1 + MAXPROJ;
  red[(rg * 128 + pn) * ns + 0] = db;
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) red[(rg * 128 + pn) * ns + 1 + q] = dw2[q];
  __syncthreads();
  if (tid < 128 && pn < a.Nr) {
    float* side = slab + (int64_t)a.Nr * Kc;
    float s = 0.f;
    for (int g2 = 0; g2 < 4; ++g2) s += red[(g2 * 128 + pn) * ns];
    side[pn] = s;
    for (int q = 0; q < a.nproj; ++q) {
      float w = 0.f;
      for (int g2 = 0; g2 < 4; ++g2) w += red[(g2 * 128 + pn) * ns + 1 + q];
      side[a.Nr + q * a.Nr + pn] = w;
    }
  }
  __syncthreads();
  // dzsum: only pn == 0 threads (one per row group) accumulated it
  if (pn == 0) {
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) red[rg * MAXPROJ + q] = dzs[q];
  }
  __syncthreads();
  if (tid < a.nproj) {
    float s = 0.f;
    for (int g2 = 0; g2 < 4; ++g2) s += red[g2 * MAXPROJ + tid];
    slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = s;
  }
}

// out[j] = Σ_b slab[b][j]   (fixed block order: deterministic)
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int64_t stride, int nblk,
                                                          float* __restrict__ out, int64_t n) {
  int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j >= n) return;
  float s = 0.0f;
  for (int b = 0; b < nblk; ++b) s += slab[(int64_t)b * stride + j];
  out[j] = s;
}

int tn_blocks(int64_t M) {
  int64_t chunks = ceil_div(M, MC);
  int64_t nb = chunks < 256 ? chunks : 256;
  return (int)(nb > 0 ? nb : 1);
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_gemm_nt_f32(const gnn_gemm_nt_params* p, gnn_stream_t stream) {
  if (!p) return fail(GNN_ERR_INVALID_ARG, __func__, "null params");
  if (p->M < 0 || p->N < 1 || p->k1 < 1 || p->k2 < 0 || !p->a1 || !p->bt || (p->k2 > 0 && !p->a2))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad shapes / null operands");
  if (p->lda1 < p->k1 || (p->k2 > 0 && p->lda2 < p->k2) || p->ldb < p->N || (p->c && p->ldc < p->N))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad leading dimensions");
  if (p->nproj < 0 || p->nproj > 4 || (p->nproj > 0 && (p->N > BN || !p->proj || !p->z || p->ldz < p->nproj)))
    return fail(GNN_ERR_INVALID_ARG, __func__, "projection needs N <= 128, nproj <= 4, proj and z");
  if (p->dropout_p < 0.f || p->dropout_p >= 1.f) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout p in [0,1)");
  if (p->M == 0) return GNN_OK;
  NTArgs a{};
  a.M = p->M; a.Nc = (int32_t)p->N;
  a.a1 = p->a1; a.lda1 = p->lda1; a.k1 = (int32_t)p->k1;
  a.a2 = p->a2; a.lda2 = p->lda2; a.k2 = (int32_t)p->k2;
  a.bt = p->bt; a.ldb = p->ldb; a.c = p->c; a.ldc = p->ldc; a.bias = p->bias; a.relu = p->relu;
  a.dropout = p->dropout_p > 0.f;
  a.keep_thresh = (uint32_t)((1.0 - (double)p->dropout_p) * 16777216.0);
  a.drop_scale = a.dropout ? (float)(1.0 / (1.0 - (double)p->dropout_p)) : 1.0f;
  a.seed = p->seed;
  a.proj = p->proj; a.nproj = p->nproj; a.z = p->z; a.ldz = p->ldz;
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  bool v4 = (a.k1 % 4 == 0) && (a.lda1 % 4 == 0) && al(a.a1, 16) &&
            (a.k2 == 0 || ((a.k2 % 4 == 0) && (a.lda2 % 4 == 0) && al(a.a2, 16)));
  bool v2 = (a.k1 % 2 == 0) && (a.lda1 % 2 == 0) && al(a.a1, 8) &&
            (a.k2 == 0 || ((a.k2 % 2 == 0) && (a.lda2 % 2 == 0) && al(a.a2, 8)));
  dim3 grid((unsigned)ceil_div(p->M, BM), (unsigned)ceil_div(p->N, BN));
  hipStream_t st = (hipStream_t)stream;
  if (v4) gemm_nt_kernel<4><<<grid, 256, 0, st>>>(a);
  else if (v2) gemm_nt_kernel<2><<<grid, 256, 0, st>>>(a);
  else gemm_nt_kernel<1><<<grid, 256, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_gemm_tn_workspace_size(int64_t M, int64_t Nr, int64_t Kc, int32_t nproj, size_t* bytes) {
  if (!bytes || M < 0 || Nr < 1 || Kc < 1 || nproj < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  int64_t stride = Nr * Kc + Nr + (int64_t)nproj * Nr + nproj;
  stride = (stride + 63) / 64 * 64;
  *bytes = (size_t)tn_blocks(M) * stride * sizeof(float);
  return GNN_OK;
}

extern "C" gnn_status gnn_gemm_tn_f32(const gnn_gemm_tn_params* p, float* out, void* workspace,
                                      size_t workspace_bytes, gnn_stream_t stream) {
  if (!p || !out) return fail(GNN_ERR_INVALID_ARG, __func__, "null params/out");
  if (p->M < 0 || p->Nr < 1 || p->Nr > 128 || p->k1 < 1 || p->k2 < 0 || p->k1 + p->k2 > KMAX)
    return fail(GNN_ERR_UNSUPPORTED, __func__, "needs 1 <= Nr <= 128 and k1 + k2 <= 384");
  if (!p->a1 || (p->k2 > 0 && !p->a2) || p->lda1 < p->k1 || (p->k2 > 0 && p->lda2 < p->k2))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad A operands");
  if (p->dz) {
    if (p->nproj < 1 || p->nproj > MAXPROJ || !p->proj || p->lddz < p->nproj)
      return fail(GNN_ERR_INVALID_ARG, __func__, "dz form needs 1 <= nproj <= 4 and proj");
  } else if (!p->g || p->ldg < p->Nr) {
    return fail(GNN_ERR_INVALID_ARG, __func__, "need g (or dz + proj)");
  }
  if (p->h && p->ldh < p->Nr) return fail(GNN_ERR_INVALID_ARG, __func__, "bad ldh");
  if (p->gout && p->ldgout < p->Nr) return fail(GNN_ERR_INVALID_ARG, __func__, "bad ldgout");
  const int32_t nproj = p->dz ? p->nproj : 0;
  const int64_t Kc = p->k1 + p->k2;
  const int64_t n_out = p->Nr * Kc + p->Nr + (int64_t)nproj * p->Nr + nproj;
  int64_t stride = (n_out + 63) / 64 * 64;
  const int nblk = tn_blocks(p->M);
  if (!workspace || workspace_bytes < (size_t)nblk * stride * sizeof(float))
    return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (p->M == 0) return hip_check(hipMemsetAsync(out, 0, n_out * sizeof(float), st), __func__);
  TNArgs a{};
  a.M = p->M; a.Nr = (int32_t)p->Nr;
  a.g = p->g; a.ldg = p->ldg; a.dz = p->dz; a.lddz = p->lddz; a.proj = p->proj; a.nproj = nproj;
  a.h = p->h; a.ldh = p->ldh; a.hscale = p->hscale;
  a.gout = p->gout; a.ldgout = p->ldgout;
  a.a1 = p->a1; a.lda1 = p->lda1; a.k1 = (int32_t)p->k1;
  a.a2 = p->a2; a.lda2 = p->lda2; a.k2 = (int32_t)p->k2;
  a.slab = static_cast<float*>(workspace); a.slab_stride = stride;
  a.rows_per_block = ceil_div(ceil_div(p->M, MC), nblk) * MC;
  gemm_tn_kernel<<<nblk, 512, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  slab_reduce_kernel<<<(unsigned)ceil_div(n_out, 256), 256, 0, st>>>(a.slab, stride, nblk, out, n_out);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
