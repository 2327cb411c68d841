// Split images ("planes") and the TN weight-gradient GEMM that reads them.
//
// The split-bf16 GEMMs (gemm_x3.hip, gemm_ws.hip) run every f32 operand as hi + mid + lo bf16
// terms.  Splitting an [N, K] operand costs ~5.5 VALU per element, and the layer-1 operand
// [agg | x] of the SAGE preset (N = 203,769, K = 332) is split twice per step (forward NT and
// backward TN) inside kernels whose MFMA phase should hide everything else: r08-r10 profiles put
// the split at ~265 of ~420 VALU per 16-row TN chunk and ~27 us of the NT.  A split image holds
// the three planes in HBM instead:
//
//   img[p][r][c]  (bf16; p = hi / mid / lo; row pitch ld; plane stride ps)
//   A1 (agg) in columns [0, k1), A2 (x) in [col2, col2 + k2), zeros elsewhere
//
// written by K1 (agg, every step: gnn_sage_mean_fwd_planes) and by gnn_split_planes_f32 (x,
// once per input tensor: x is a constant of the training run, like the CSR plan).  The GEMMs then
// stage A by plain 16-byte copies: 6 B per element instead of 4 B, no split instructions.
//
// TN (this file): dW = Gᵀ·[A1 | A2] over 16-row chunks (one MFMA k-step).  The chunk's three
// A planes are copied as rows into LDS ([plane][16 rows][352], 704-byte pitch ≡ 48 dwords mod
// 64) and read as the MFMA B operand by ds_read_b64_tr_b16 (a 16-lane group reads 4 rows x 16
// columns and receives them column-major: two reads give a lane its 8 consecutive rows of one
// column, conflict-free at this pitch).  G is formed and split on the fly as in gemm_x3.hip.
#include "gemm_common.hpp"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef float f32x2v_t __attribute__((ext_vector_type(2)));

namespace gnnmp {
namespace {

// ------------------------------------------------------------------ split image of an f32 matrix
// One thread per column pair of one row: hi / mid / lo words of the pair (zeros at columns >= F).
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                           int32_t F, uint16_t* __restrict__ img, int64_t ld,
                                                           int64_t ps, int32_t width) {
  const int hw = width >> 1;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * hw) return;
  const int64_t r = i / hw;
  const int c = 2 * (int)(i - r * hw);
  const float* xr = x + r * ldx;
  const float a = c < F ? xr[c] : 0.0f;
  const float b = c + 1 < F ? xr[c + 1] : 0.0f;
  uint32_t h, m, l;
  split3_pair(a, b, h, m, l);
  uint32_t* d = reinterpret_cast<uint32_t*>(img + r * ld + c);
  d[0] = h;
  d[ps >> 1] = m;
  d[ps] = l;
}

// half-pair image of an f32 matrix pre-scaled by the power of two s (exact): one thread per column
// pair of one row (zeros at columns >= F)
__global__ __launch_bounds__(256) void split_h2_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                       int32_t F, uint16_t* __restrict__ img, int64_t ld, int64_t ps,
                                                       int32_t width, float s) {
  const int hw = width >> 1;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * hw) return;
  const int64_t r = i / hw;
  const int c = 2 * (int)(i - r * hw);
  const float* xr = x + r * ldx;
  const float a = c < F ? xr[c] * s : 0.0f;
  const float b = c + 1 < F ? xr[c + 1] * s : 0.0f;
  uint32_t h, l;
  split_h2_pair(a, b, h, l);
  uint32_t* d = reinterpret_cast<uint32_t*>(img + r * ld + c);
  d[0] = h;
  d[ps >> 1] = l;
}

// ------------------------------------------------------------------ TN over a split image
constexpr int PT_ROWS = 16;               // rows per chunk = one MFMA k-step
constexpr int PT_AP = 352;                // LDS row pitch of an A chunk (bf16): 704 B ≡ 48 dwords mod 64
constexpr int PT_APL = PT_ROWS * PT_AP;   // one plane of a chunk
constexpr int PT_GP = 24;                 // G row pitch ([n][m], 12 dwords: conflict-free b128 reads)
constexpr int PT_GPL = 128 * PT_GP;
// 16-byte A pieces per thread per chunk: 8 at 256 threads, 4 at 512 (3·16·42 = 2016 <= 2048)
constexpr int PT_MAXLD = 336;             // widest image row the chunk layout holds (42 pieces)

// one transposed 4-row x 16-column read (lane i of each 16-lane group gets column i)
__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat_frag(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Block: 4 waves (one per SIMD); wave w owns dW rows 32w .. +32 (G columns) x all KT k-tiles of
// the image width.  Rows: blockIdx.x·rows_per_block .. in chunks of 16, each LOADED from row
// min(start, M - 16) so every load is in bounds (the G mask zeroes rows outside the block).
// Software-pipelined: iteration c runs chunk c's 6·KT MFMAs and, between them (sched_barrier
// fences pin the order), stages chunk c+1 into the other LDS buffers in 22 units — per thread
// PT_NP A pieces (one ds_write_b128 each, then the refill load of chunk c+2), one G slot
// (column n = tid mod 128, 8 consecutive rows: G = (dz·P) ⊙ mask or g ⊙ mask, split, 3
// ds_write_b128) and the dz ring slot of chunk c+2.  One barrier per chunk.  With one wave per
// SIMD the staging issues in the MFMAs' shadow instead of in a phase of its own.
// LAB (timing ablations, csrc/lab/lab_tn.hip only; the library instantiates 0): bit 1 no MFMAs,
// bit 2 no staging slots, bit 4 no fragment reads in the loop, bit 8 no per-chunk barrier.
// KS = 2 (Nr <= 64): waves 0-1 own dW rows 0..63 over the first half of the k-tiles, waves 2-3
// the same rows over the second half (each dW element still one wave's chain: same results), so
// no wave multiplies the zero G columns 64..127 and the MFMA chain the staging hides behind halves.
// NW = 8 (r19): two waves per SIMD, the k-tiles split KS ways over RG = NW / KS row groups (as
// evenly as KT allows: wave group kg owns tiles [kg·KT/KS, (kg+1)·KT/KS)), twice the staging threads.
template <bool PROJ, bool MASK, int KT, bool GOUT, int LAB = 0, int KS = 1, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemm_tn_planes_kernel(TNArgs a) {
  constexpr int RG = NW / KS;  // row groups of 32 dW rows
  static_assert((NW == 4 || NW == 8) && (RG == 2 || RG == 4) && RG * KS == NW, "wave layout");
  constexpr bool EVEN = KT % KS == 0;
  constexpr int KW = (KT + KS - 1) / KS;  // k-tiles per wave (at most)
  constexpr int T = 64 * NW;
  constexpr int NP = (3 * PT_ROWS * (PT_MAXLD / 8) + T - 1) / T;  // A pieces per thread (8 / 4)
  constexpr int RP = PT_ROWS / (T / 128);                          // G rows per thread (8 / 4)
  __shared__ __attribute__((aligned(16))) uint16_t Gt[2][3 * PT_GPL];
  __shared__ __attribute__((aligned(16))) uint16_t At[2][3 * PT_APL];
  __shared__ float dzL[2][256];  // dz rows of a chunk (16 x 4), threads 0..63 write theirs
  constexpr int NU = 2 * NP + RP / 2 + 2 * RP + RP + 3;  // staging slots per chunk (47 / 25)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ld = a.ap_ld;
  const int pr = ld >> 3;  // 16-byte pieces per image row
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);
  const int nch = mend > mbeg ? (int)((mend - mbeg + PT_ROWS - 1) / PT_ROWS) : 0;

  const int wr = wave % RG;                          // the wave's 32 dW rows
  const int kg = wave / RG;                          // its k-tile group
  const int t0 = kg * KT / KS;                       // first k-tile
  const int ntl = (kg + 1) * KT / KS - t0;           // and count (KW when EVEN)
  floatx16 acc[KW];
#pragma unroll
  for (int t = 0; t < KW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  // ---- A pieces of this thread (chunk-invariant): byte offsets in the image (relative to the
  //      chunk's first row) and in the LDS chunk.  Idle pieces re-load piece 0 into a pad slot
  //      (columns 336.. of plane 0, never part of a written dW column).
  const __amdgpu_buffer_rsrc_t arsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.ap), 0, (int)(3 * a.ap_ps * 2), 0x00020000);
  uint32_t goff[NP], loff[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int q = tid + T * j;
    const int per_plane = PT_ROWS * pr;
    const bool ok = q < 3 * per_plane;
    const int p = q / per_plane, rr = q - p * per_plane;
    const int row = rr / pr, c16 = rr - row * pr;
    goff[j] = ok ? (uint32_t)(((int64_t)p * a.ap_ps + (int64_t)row * ld + 8 * c16) * 2) : 0u;
    loff[j] = ok ? (uint32_t)((p * PT_APL + row * PT_AP + 8 * c16) * 2)
                 : (uint32_t)(((tid & 15) * PT_AP + PT_MAXLD + 8 * ((tid >> 4) & 1)) * 2);
  }

  // ---- G slot: column gn, rows RP·go .. +RP of the chunk
  const int gn = tid & 127, go = tid >> 7;
  const bool gcol = gn < a.Nr;
  const int gnc = gcol ? gn : 0;
  const float* gbase = MASK ? a.h + gnc : a.g + gnc;
  const int gld = MASK ? (int)a.ldh : (int)a.ldg;
  const float* g2base = a.g + gnc;  // the g form with MASK: g values beside h
  const int g2ld = (int)a.ldg;
  const int zr = (tid & 63) / MAXPROJ, zq = (tid & 63) % MAXPROJ;
  const int zqc = PROJ ? min(zq, a.nproj - 1) : 0;
  float pcol[MAXPROJ];
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) pcol[q] = (PROJ && q < a.nproj && gcol) ? a.proj[q * a.Nr + gn] : 0.0f;

  const int Mi = (int)a.M;
  auto ldbase = [&](int c) { return min((int)mbeg + c * PT_ROWS, Mi - PT_ROWS); };
  const int clast = max(nch - 1, 0);
  u32x4 ra[NP];
  float rg[RP], rg2[RP];
  float rz = 0.f;
  // loads of chunk c into the stage registers (c clamped by the callers: always in bounds)
  auto load_a = [&](int j, int c) {
    ra[j] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)goff[j], ldbase(c) * ld * 2, 0);
  };
  auto load_g = [&](int c) {
    const int mb = ldbase(c);
    if constexpr (MASK || !PROJ) {  // the dz form without a mask reads no G column
      uint32_t o = (uint32_t)((mb + RP * go) * gld);
#pragma unroll
      for (int i = 0; i < RP; ++i) {
        rg[i] = gbase[o];
        o += (uint32_t)gld;
      }
    }
    if constexpr (MASK && !PROJ) {
      uint32_t o2 = (uint32_t)((mb + RP * go) * g2ld);
#pragma unroll
      for (int i = 0; i < RP; ++i) {
        rg2[i] = g2base[o2];
        o2 += (uint32_t)g2ld;
      }
    }
  };
  auto load_z = [&](int c) {
    if constexpr (PROJ) rz = a.dz[(uint32_t)((ldbase(c) + zr) * (int)a.lddz + zqc)];
  };
  // the dz ring slot of chunk k (zero outside the block's rows: G, dzᵀh and Σdz need no row masks)
  auto put_z = [&](int k) {
    if constexpr (PROJ) {
      const int mb = ldbase(k);
      const bool ok = tid < PT_ROWS * MAXPROJ && zq < a.nproj && zr >= (int)mbeg + k * PT_ROWS - mb &&
                      zr < (int)mend - mb;
      if (T == 256 || tid < 256) dzL[k & 1][tid] = ok ? rz : 0.0f;
    }
  };

  float db = 0.f, dzs = 0.f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float e[RP];
  uint32_t w[RP / 2][3];
  float4 zv[RP];  // dz rows of the G slot (read in one unit, ahead of their use)
  float zsv[RP];
  auto z_read = [&](int c, int i0, int n) {  // rows i0 .. i0 + n of the G slot
    if constexpr (PROJ) {
      const int buf = c & 1;
#pragma unroll
      for (int i = i0; i < i0 + n; ++i) {
        const int r = RP * go + i;
        zv[i] = *reinterpret_cast<const float4*>(&dzL[buf][r * MAXPROJ]);
        zsv[i] = dzL[buf][r * MAXPROJ + (gn & (MAXPROJ - 1))];
      }
    }
  };
  auto put_a = [&](int j, int c) {
    *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(At[c & 1]) + loff[j]) = ra[j];
  };
  // G row i of the slot (after z_read), in two halves (e[i] carries the raw value between them)
  auto g_row = [&](int i, int c, int half) {
    if (half == 0) {
      if constexpr (PROJ) {
        const float4 z = zv[i];
        float g = z.x * pcol[0];
        g = fmaf(z.y, pcol[1], g);
        g = fmaf(z.z, pcol[2], g);
        e[i] = fmaf(z.w, pcol[3], g);
        if constexpr (MASK) {
          dw2[0] = fmaf(z.x, rg[i], dw2[0]);
          dw2[1] = fmaf(z.y, rg[i], dw2[1]);
          dw2[2] = fmaf(z.z, rg[i], dw2[2]);
          dw2[3] = fmaf(z.w, rg[i], dw2[3]);
        }
      } else {
        e[i] = MASK ? rg2[i] : rg[i];
      }
      return;
    }
    const int mb = ldbase(c);
    const int r = RP * go + i;
    const bool ok = r >= (int)mbeg + c * PT_ROWS - mb && r < (int)mend - mb && gcol;
    float g = e[i];
    if constexpr (PROJ) dzs += gn < MAXPROJ ? zsv[i] : 0.0f;  // unconditional read + select: no branch
    if constexpr (MASK) g = rg[i] > 0.0f ? g * a.hscale : 0.0f;
    if constexpr (!PROJ) g = ok ? g : 0.0f;
    db += g;
    if constexpr (GOUT) {
      if (a.gout && ok) a.gout[(int64_t)(mb + r) * a.ldgout + gn] = g;
    }
    e[i] = g;
  };
  // split3_pair of (e[2j], e[2j+1]) in two halves: hi and the first remainders, then mid / lo
  auto split_half = [&](int j, int half) {
    typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
    typedef float f32x2_ __attribute__((ext_vector_type(2)));
    float& x0 = e[2 * j];
    float& x1 = e[2 * j + 1];
    if (half == 0) {
      const uint32_t h = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{x0, x1}, bf16x2_));
      w[j][0] = h;
      x0 -= __uint_as_float(h << 16);
      x1 -= __uint_as_float(h & 0xffff0000u);
    } else {
      const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{x0, x1}, bf16x2_));
      w[j][1] = m;
      const float y0 = x0 - __uint_as_float(m << 16);
      const float y1 = x1 - __uint_as_float(m & 0xffff0000u);
      w[j][2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{y0, y1}, bf16x2_));
    }
  };
  auto g_put = [&](int c) {
    uint16_t* gd = Gt[c & 1] + gn * PT_GP + RP * go;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if constexpr (RP == 8) *reinterpret_cast<uint4*>(gd + p * PT_GPL) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
      else *reinterpret_cast<uint2*>(gd + p * PT_GPL) = make_uint2(w[0][p], w[1][p]);
    }
  };
  // staging slot k of chunk c + 1, issued right after one MFMA of chunk c (a few instructions in
  // the MFMA's shadow); refills for chunks c + 2 / c + 3
  auto unit = [&](int k, int c) {
    constexpr int A0 = 0, Z0 = 2 * NP, G0 = Z0 + RP / 2, S0 = G0 + 2 * RP, P0 = S0 + RP;
    if (k < Z0) {
      if (k & 1) load_a(k >> 1, min(c + 2, clast));
      else put_a(k >> 1, c + 1);
    } else if (k < G0) {
      z_read(c + 1, 2 * (k - Z0), 2);
    } else if (k < S0) {
      g_row((k - G0) >> 1, c + 1, (k - G0) & 1);
    } else if (k < P0) {
      split_half((k - S0) >> 1, (k - S0) & 1);
    } else if (k == P0) {
      g_put(c + 1);
    } else if (k == P0 + 1) {
      load_g(min(c + 2, clast));
    } else if (k == P0 + 2) {
      put_z(c + 2);
      load_z(min(c + 3, clast));
    }
    (void)A0;
  };
  static_assert(2 * NP + RP / 2 + 2 * RP + RP + 3 == NU, "slot count");

  // fragment addresses: G rows 32·wave + (lane & 31), k = 8·(lane >> 5); A (transposed reads)
  // lane 4q + p of 16-lane group g supplies row 8·(g >> 1) + q, columns 16·(g & 1) + 4p ..
  const int gfo = (32 * wr + (lane & 31)) * PT_GP + 8 * (lane >> 5);
  const int grp = lane >> 4, li = lane & 15;
  const int afo = (8 * (grp >> 1) + (li >> 2)) * PT_AP + 16 * (grp & 1) + 4 * (li & 3);
  auto afrag = [&](const uint16_t* base, int t, int p) {
    const uint16_t* q = base + p * PT_APL + t * 32;
    return cat_frag(tr_read(q), tr_read(q + 4 * PT_AP));
  };
#define PT_FENCE __builtin_amdgcn_sched_barrier(0)
  auto compute = [&](int c) {
    const int buf = c & 1;
    bf16x8 gf[3], af[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) gf[p] = *reinterpret_cast<const bf16x8*>(Gt[buf] + p * PT_GPL + gfo);
    const uint16_t* ab = At[buf] + afo;
#pragma unroll
    for (int p = 0; p < 3; ++p) af[0][p] = afrag(ab, t0, p);
    // tile t+1's fragment reads are issued before tile t's MFMAs (in flight across them); one
    // staging slot after each MFMA (fences pin the order: the slot issues in the MFMA's shadow)
    constexpr int pa[6] = {1, 2, 0, 1, 0, 0}, pb[6] = {1, 0, 2, 0, 1, 0};  // small terms first
#pragma unroll
    for (int t = 0; t < KW; ++t) {
      if (t + 1 < KW && !(LAB & 4)) {
#pragma unroll
        for (int p = 0; p < 3; ++p) af[(t + 1) & 1][p] = afrag(ab, t0 + t + 1, p);
      }
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        PT_FENCE;
        if constexpr (!(LAB & 1)) {
          if (EVEN || t < ntl)  // wave-uniform
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[pa[m]], af[(LAB & 4) ? 0 : (t & 1)][pb[m]], acc[t], 0, 0, 0);
        }
        PT_FENCE;
        if (6 * t + m < NU && !(LAB & 2)) unit(6 * t + m, c);
      }
      PT_FENCE;
    }
#pragma unroll
    for (int u = 6 * KW; u < NU; ++u)  // narrow images: the slots past the MFMAs
      if (!(LAB & 2)) unit(u, c);
    if constexpr ((LAB & 1) != 0) {  // keep the fragments live
#pragma unroll
      for (int t = 0; t < KW; ++t) acc[t][0] += (float)gf[0][0] + (float)af[0][0][0] + (float)af[1][1][1];
    }
  };
#undef PT_FENCE

  if (nch > 0) {
    // prologue: dz ring slots of chunks 0 and 1, chunk 0 staged directly, chunk 1 and dz(2) loaded
    rz = PROJ ? a.dz[(uint32_t)((ldbase(0) + zr) * (int)a.lddz + zqc)] : 0.f;
    put_z(0);
    load_z(min(1, clast));
    put_z(1);
    load_z(min(2, clast));
#pragma unroll
    for (int j = 0; j < NP; ++j) load_a(j, 0);
    load_g(0);
    __syncthreads();  // dzL
#pragma unroll
    for (int j = 0; j < NP; ++j) put_a(j, 0);
    z_read(0, 0, RP);
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      g_row(i, 0, 0);
      g_row(i, 0, 1);
    }
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) split3_pair(e[2 * j], e[2 * j + 1], w[j][0], w[j][1], w[j][2]);
    g_put(0);
#pragma unroll
    for (int j = 0; j < NP; ++j) load_a(j, min(1, clast));
    load_g(min(1, clast));
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      compute(c);       // + staging of chunk c + 1 into the other buffers (read by chunk c - 1:
      if constexpr (!(LAB & 8)) __syncthreads();  //   retired by the previous barrier)
    }
  }

  // ---- this block's partial dW (segment-major: dW1 = [Nr][k1] then dW2 = [Nr][k2])
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  const int Kc = a.k1 + a.k2;
#pragma unroll
  for (int t = 0; t < KW; ++t) {
    if (!EVEN && t >= ntl) break;  // wave-uniform
    const int kp = (t0 + t) * 32 + (lane & 31);  // image column
    const bool s1 = kp < a.k1;
    const bool s2 = kp >= a.ap_col2 && kp < a.ap_col2 + a.k2;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t idx = s1 ? (int64_t)row * a.k1 + kp : (int64_t)a.Nr * a.k1 + (int64_t)row * a.k2 + (kp - a.ap_col2);
      if (row < a.Nr && (s1 || s2)) slab[idx] = acc[t][r];
    }
  }
  __syncthreads();
  // side sums of the two row octets combined in a fixed order through LDS (At[0] is free now)
  float* red = reinterpret_cast<float*>(&At[0][0]);
  constexpr int ns = 2 + MAXPROJ;
  red[(go * 128 + gn) * ns + 0] = db;
  red[(go * 128 + gn) * ns + 1] = dzs;
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) red[(go * 128 + gn) * ns + 2 + q] = dw2[q];
  __syncthreads();
  constexpr int NGO = T / 128;  // row groups of a column, combined in order
  auto comb = [&](int col, int f) {
    float v = red[col * ns + f];
#pragma unroll
    for (int o = 1; o < NGO; ++o) v += red[(o * 128 + col) * ns + f];
    return v;
  };
  if (tid < 128 && tid < a.Nr) {
    float* side = slab + (int64_t)a.Nr * Kc;
    side[tid] = comb(tid, 0);
    for (int q = 0; q < a.nproj; ++q) side[a.Nr + q * a.Nr + tid] = comb(tid, 2 + q);
  }
  if (PROJ && tid < a.nproj) slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = comb(tid, 1);
}

// (ABI 26) dz[r, 0:ccols] = Σ_{CSC slots s of row r} u[row[s], :] for the rows [mbeg, mend) of a
// TN block — gnn_aggregate_f32(SUM, transpose) of u, i.e. aggregate.hip's agg_narrow_lds_kernel
// <SUM, NF = 2, 256, COOP> restated for the TN's waves, bit for bit: the same 64-row groups (aligned
// as that kernel's waves), the same 256-slot LDS passes from the group's first slot, the same four
// interleaved partial sums per lane and the same whole-wave xor tree for slots past the first 32 of
// a pass.  Wave w of the block takes groups w, w + NW, ...; a lane stores only its block's rows.
// `buf`: 512 floats of LDS per wave.  The block's whole dz rows (the folded columns and the ones
// read, q < nproj) also go to `dzb` ([row - mbeg][MAXPROJ], LDS), where the prologue's first two
// chunks read them instead of a round trip to dz, and the return value is the lane's part of the
// block scale's bound: max over its rows of Σ_q |dz[r][q]| in the scan's own order.
template <int NW>
__device__ __forceinline__ float tn_csc_fold(const TNArgs& a, int64_t mbeg, int64_t mend, float* buf, float* dzb,
                                             int lane, int wave) {
  constexpr int CAP = 256, NI = CAP / 64, LCAP = 32;
  const int F = a.ccols, nq = a.nproj;
  const int64_t nrows = a.M;
  float* dz = const_cast<float*>(a.dz);
  float zm = 0.f;
  for (int64_t r0 = ((mbeg >> 6) + wave) * 64; r0 < mend; r0 += 64 * NW) {
    const int64_t r = r0 + lane;
    const bool rok = r < nrows;
    const int32_t pbeg = a.cptr[rok ? r : nrows];
    const int32_t pend = a.cptr[rok ? r + 1 : nrows];
    const int32_t base = __builtin_amdgcn_readfirstlane(a.cptr[r0]);
    const int32_t wend = __builtin_amdgcn_readfirstlane(a.cptr[min(r0 + 64, nrows)]);
    float dv[MAXPROJ];  // the row's columns past the folded ones (clamped row / column, no branch)
    const int64_t rc = min(r, nrows - 1);
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) dv[q] = a.dz[rc * a.lddz + min(max(q, F), nq - 1)];
    float acc[2] = {0.f, 0.f};
    for (int32_t pb = base; pb < wend; pb += CAP) {
      const int32_t pe = min(pb + CAP, wend);
      int32_t nn[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int32_t k = pb + lane + 64 * i;
        nn[i] = a.cnbr[k < pe ? k : pb];
      }
      float xv[NI][2];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float* xr = a.cu + (int64_t)nn[i] * a.ldu;
#pragma unroll
        for (int f = 0; f < 2; ++f) xv[i][f] = xr[f < F ? f : 0];
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int f = 0; f < 2; ++f) buf[f * CAP + lane + 64 * i] = f < F ? xv[i][f] : 0.0f;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      const int32_t lo = max(pbeg, pb), hi0 = min(pend, pe);
      const int32_t hi = min(hi0, lo + LCAP);
      float q1[2] = {0.f, 0.f}, q2[2] = {0.f, 0.f}, q3[2] = {0.f, 0.f};
      int32_t k = lo;
      for (; k + 3 < hi; k += 4) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          acc[f] += buf[f * CAP + (k - pb)];
          q1[f] += buf[f * CAP + (k + 1 - pb)];
          q2[f] += buf[f * CAP + (k + 2 - pb)];
          q3[f] += buf[f * CAP + (k + 3 - pb)];
        }
      }
      for (; k < hi; ++k) {
#pragma unroll
        for (int f = 0; f < 2; ++f) acc[f] += buf[f * CAP + (k - pb)];
      }
#pragma unroll
      for (int f = 0; f < 2; ++f) acc[f] += (q1[f] + q2[f]) + q3[f];
      uint64_t longm = __ballot(hi0 - lo > LCAP);  // the rest of each long row: all 64 lanes, strided
      while (longm) {
        const int L = __builtin_ctzll(longm);
        longm &= longm - 1;
        const int32_t s0 = __builtin_amdgcn_readlane(lo, L) + LCAP, s1 = __builtin_amdgcn_readlane(hi0, L);
        float part[2] = {0.f, 0.f};
        for (int32_t k2 = s0 + lane; k2 < s1; k2 += 64) {
#pragma unroll
          for (int f = 0; f < 2; ++f) part[f] += buf[f * CAP + (k2 - pb)];
        }
#pragma unroll
        for (int f = 0; f < 2; ++f) {
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) part[f] += __shfl_xor(part[f], off);
          if (lane == L) acc[f] += part[f];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (rok && r >= mbeg && r < mend) {
#pragma unroll
      for (int f = 0; f < 2; ++f)
        if (f < F) dz[r * a.lddz + f] = acc[f];
      float v[MAXPROJ];
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) v[q] = q == 0 ? acc[0] : (q == 1 && F > 1) ? acc[1] : dv[q];
      float sr = 0.f;  // (the scan's Σ_q |dz[r][q]|, same order)
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) {
        sr += q < nq ? fabsf(v[q]) : 0.f;
        dzb[(r - mbeg) * MAXPROJ + q] = v[q];
      }
      zm = fmaxf(zm, sr);
    }
  }
  return zm;
}

// ------------------------------------------------------------------ TN over a half-pair image
// dW = Gᵀ·[A1 | A2] with A from a half-pair image (2 f16 planes hi / lo, gemm_ws.hip K7a-h) and
// G — the dz form with the h mask, G = (dz·P) ⊙ [h > 0] / (1 - p), the SAGE preset's hidden
// layer — formed on the fly, scaled by this block's power of two s_b (|G·s_b| < 16: the bound
// hscale · max_rows Σ_q |dz_q| · max |P| over the block's rows, one pass over its dz rows before
// the chunk loop) and held as three f16 planes hi' = 2^11 hi, hi, lo.  Three products per k-tile
// into one accumulator (the split-image kernel above runs six):
//     acc += G_hi'·A_hi + G_lo·A_hi + G_hi·A_lo  (= 2^11 s_b · Gᵀ·A up to 2^-22 relative)
// and the slab gets acc · 2^-11 / s_b (exact; also / 2^ap_exp, the A image's pre-scale).  The side sums (Σ G, dzᵀ·h, Σ dz) are f32 sums of
// the unscaled values, as in the split-image kernel.  Geometry, the chunk pipeline and slab
// layout are the split-image kernel's: 4 waves, wave w owns dW rows 32w .. +32 x all KT k-tiles,
// 16-row chunks, one barrier per chunk, the staging of chunk c+1 spread over chunk c's 3·KT MFMA
// gaps (several units per gap).  LAB as above (bit 1 no MFMAs, 2 no staging, 4 no fragment reads).
// NW = 8 (r19): two waves per SIMD — waves w and w + 4 share dW rows 32(w & 3) .. +32 and split the
// k-tiles (the first (KT + 1) / 2 and the rest), so each holds half the accumulators and the block
// twice the staging threads (twice the chunk loads in flight per CU).
// GF (round 5): the plain g form — G = g read as is ([M, Nr] f32: the input layer's weight
// gradient of GCN / GAT layer 1 and of SAGE-ResBN layer 0's conv and residual projection, dW =
// Gᵀ·x over x's half-pair image), block scale from max |g| over the block's rows (one pass over
// them before the chunk loop, behind chunk 0's loads), side sums: db = Σ G only.
// KS = 2 (round 6, strong-scaling shards): split-K across block pairs — blocks 2b and 2b + 1 take
// the same rows and the first (KT + 1) / 2 / the remaining k-tiles, so a shard-sized M runs twice
// the rows per block on every CU and writes half the slab partials (both blocks form the same G;
// the side sums come from the first).  The block's A pieces cover only its k-range.
// CSC (round 6, ABI 26; the dz form): the block first forms dz[:, 0:ccols] of its own rows — the
// transposed mean of the output layer, Σ over each row's CSC slots of u[src] (u = dlogits / deg
// from the CE launch) — with tn_csc_fold below, writes them to dz and reads them back as before:
// the separate F = 2 CSC-sum launch of the step is gone.
template <int KT, bool GOUT, int LAB = 0, int NW = 4, bool GF = false, int KS = 1, bool CSC = false>
__global__ __launch_bounds__(64 * NW) void gemm_tn_h2_kernel(TNArgs a) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(KS == 1 || (KS == 2 && NW == 8), "split-K: the 8-wave form");
  constexpr int T = 64 * NW;
  constexpr int NPA = (2 * PT_ROWS * (PT_MAXLD / 8) + T - 1) / T;  // A pieces per thread per chunk (6 / 3)
  constexpr int RP = PT_ROWS / (T / 128);                           // G rows per thread per chunk (8 / 4)
  constexpr int KTB = KS == 1 ? KT : (KT + 1) / 2;                   // k-tiles of a block (at most)
  constexpr int KTW = NW == 4 ? KTB : (KTB + 1) / 2;                // k-tiles per wave
  __shared__ __attribute__((aligned(16))) uint16_t Gt[2][3 * PT_GPL];
  __shared__ __attribute__((aligned(16))) uint16_t At[2][2 * PT_APL];
  __shared__ float dzL[2][256];
  __shared__ float redm[2 * NW];
  constexpr int NU = 2 * NPA + RP / 2 + 2 * RP + RP / 2 + 3;  // staging units per chunk
  constexpr int NG = 3 * KTW;                                 // MFMA gaps per chunk
  // A's register ring: RING sets of the NPA pieces, a chunk's loads issued RING chunks before
  // its LDS put.  LAB 16: two sets — measured slower (lab 104.2 vs 100.6 us, r18h: the second
  // set's 24 VGPRs cost more in the chunk loop than the extra lead buys)
  constexpr int RING = (LAB & 16) ? 2 : 1;
  // RGN: register sets of G rows (2: two chunks ahead; measured no faster on the g form, r27: 70.0
  // vs 66.9 us on the GCN layer-1 shape, so one set)
  constexpr int RGN = 1;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ld = a.ap_ld;
  const int kpart = KS == 1 ? 0 : (int)(blockIdx.x & 1);   // split-K: this block's k-range
  const int rblk = KS == 1 ? (int)blockIdx.x : (int)(blockIdx.x >> 1);
  const int kt0 = kpart * KTB;                              // first k-tile
  const int ktb = KS == 1 ? KT : (kpart ? KT - KTB : KTB);  // k-tiles of this block
  const int pr = min(4 * ktb, (ld - 32 * kt0) >> 3);        // 16-byte A pieces per row
  const int64_t mbeg = (int64_t)rblk * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);
  const int nch = mend > mbeg ? (int)((mend - mbeg + PT_ROWS - 1) / PT_ROWS) : 0;
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  const int wrow = 32 * (wave & 3);                             // this wave's dW rows
  const int tbase = NW == 4 ? 0 : (wave >> 2) * KTW;            // and k-tiles [tbase, tbase + ntl) of the block
  const int ntl = NW == 4 ? KT : max(0, min(KTW, ktb - tbase));

  floatx16 acc[KTW];
#pragma unroll
  for (int t = 0; t < KTW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  const __amdgpu_buffer_rsrc_t arsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.ap), 0, (int)(2 * a.ap_ps * 2), 0x00020000);
  uint32_t goff[NPA], loff[NPA];
#pragma unroll
  for (int j = 0; j < NPA; ++j) {
    const int q = tid + T * j;
    const int per_plane = PT_ROWS * pr;
    const bool ok = q < 2 * per_plane;
    const int p = q / per_plane, rr = q - p * per_plane;
    const int row = rr / pr, c16 = rr - row * pr;
    goff[j] = ok ? (uint32_t)(((int64_t)p * a.ap_ps + (int64_t)row * ld + 32 * kt0 + 8 * c16) * 2) : 0u;
    loff[j] = ok ? (uint32_t)((p * PT_APL + row * PT_AP + 8 * c16) * 2)
                 : (uint32_t)(((tid & 15) * PT_AP + PT_MAXLD + 8 * ((tid >> 4) & 1)) * 2);
  }

  // ---- G slot: column gn, rows RP·go .. +RP of the chunk
  const int gn = tid & 127, go = tid >> 7;
  const bool gcol = gn < a.Nr;
  const int gnc = gcol ? gn : 0;
  const float* hb = GF ? a.g + gnc : a.h + gnc;  // the g form loads G itself where the dz form loads h
  const int hld = GF ? (int)a.ldg : (int)a.ldh;
  const int zr = (tid & 63) / MAXPROJ, zq = (tid & 63) % MAXPROJ;
  const int zqc = min(zq, a.nproj - 1);
  float pcol[MAXPROJ];
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) pcol[q] = (!GF && q < a.nproj && gcol) ? a.proj[q * a.Nr + gn] : 0.0f;

  // ---- the block's G scale s_b: |G| <= hscale · max_m Σ_q |dz[m][q]| · max |P|.  The dz rows are
  // read 4 per thread per pass with clamped indices and no branch around a load, so a pass is one
  // round trip (the first form's per-row loop waited on every row: ~5 us of the prologue)
  float gsc = 1.f, gunsc = 1.f;
  float zm_fold = 0.f;  // CSC: the fold's part of the bound (the scan then reads no dz rows)
  auto scan_scale = [&]() __attribute__((always_inline)) {  // run in the prologue, behind chunk 0's loads
    float zm = zm_fold;
    const int nq = a.nproj;
    if (GF && a.growmax) {  // (ABI 25) the producer's row-group maxima: ~50 words, not ~800 rows
      const int64_t q1 = (mend + GNN_ROWMAX_ROWS - 1) / GNN_ROWMAX_ROWS;
      for (int64_t q = mbeg / GNN_ROWMAX_ROWS + tid; q < q1; q += T) zm = fmaxf(zm, __uint_as_float(a.growmax[q]));
    } else if constexpr (GF) {  // max |g| over the block's rows: float4 pieces, 16 in flight per thread
      constexpr int SU = 16;  // (the block's ~800 rows in two round trips: the scan is latency-bound)
      const int n4 = (a.Nr + 3) >> 2;
      const int64_t npc = (mend - mbeg) * n4;
      for (int64_t q0 = tid; q0 < npc; q0 += SU * T) {
        float4 v[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int64_t q = min(q0 + (int64_t)T * u, npc - 1);
          const int64_t r = mbeg + q / n4;
          const int c4 = (int)(q - (q / n4) * n4) * 4;
          v[u] = *reinterpret_cast<const float4*>(a.g + r * a.ldg + c4);
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int64_t q = q0 + (int64_t)T * u;
          const int c4 = (int)(min(q, npc - 1) % n4) * 4;  // columns past Nr (the last piece) masked
          float m = fabsf(v[u].x);
          m = fmaxf(m, c4 + 1 < a.Nr ? fabsf(v[u].y) : 0.f);
          m = fmaxf(m, c4 + 2 < a.Nr ? fabsf(v[u].z) : 0.f);
          m = fmaxf(m, c4 + 3 < a.Nr ? fabsf(v[u].w) : 0.f);
          zm = fmaxf(zm, q < npc ? m : 0.f);
        }
      }
    }
    for (int64_t r0 = mbeg + tid; !GF && !CSC && r0 < mend; r0 += 4 * T) {
      float v[4][MAXPROJ];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t r = min(r0 + (int64_t)T * u, mend - 1);
#pragma unroll
        for (int q = 0; q < MAXPROJ; ++q) v[u][q] = a.dz[r * a.lddz + min(q, nq - 1)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < MAXPROJ; ++q) s += q < nq ? fabsf(v[u][q]) : 0.f;
        zm = fmaxf(zm, r0 + (int64_t)T * u < mend ? s : 0.f);
      }
    }
    float pm = 0.f;
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) pm = fmaxf(pm, fabsf(pcol[q]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      zm = fmaxf(zm, __shfl_xor(zm, o));
      pm = fmaxf(pm, __shfl_xor(pm, o));
    }
    if (lane == 0) {
      redm[wave] = zm;
      redm[NW + wave] = pm;
    }
    __syncthreads();
    zm = redm[0];
    pm = redm[NW];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      zm = fmaxf(zm, redm[w]);
      pm = fmaxf(pm, redm[NW + w]);
    }
    const float bound = GF ? zm : zm * pm * a.hscale;
    int E = 0;
    if (bound > 0.f && isfinite(bound)) frexpf(bound, &E);  // bound < 2^E
    gsc = ldexpf(1.0f, 4 - E);                               // |G · gsc| < 16
    gunsc = ldexpf(1.0f, E - 4 - 11 - a.ap_exp);             // slab = acc · 2^-11 / gsc / 2^ap_exp
  };

  const int Mi = (int)a.M;
  auto ldbase = [&](int c) __attribute__((always_inline)) { return min((int)mbeg + c * PT_ROWS, Mi - PT_ROWS); };
  const int clast = max(nch - 1, 0);
  u32x4 ra[RING][NPA];
  float rg[RGN][RP];
  float rz = 0.f;
  auto load_a = [&](int s, int j, int c) __attribute__((always_inline)) {
    ra[s][j] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)goff[j], ldbase(c) * ld * 2, 0);
  };
  auto load_g = [&](int sg, int c) __attribute__((always_inline)) {
    uint32_t o = (uint32_t)((ldbase(c) + RP * go) * hld);
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      rg[sg][i] = hb[o];
      o += (uint32_t)hld;
    }
  };
  auto load_z = [&](int c) __attribute__((always_inline)) {
    if constexpr (!GF) rz = a.dz[(uint32_t)((ldbase(c) + zr) * (int)a.lddz + zqc)];
  };
  auto put_zv = [&](int k, float v) __attribute__((always_inline)) {
    if constexpr (GF) return;
    const int mb = ldbase(k);
    const bool ok = tid < PT_ROWS * MAXPROJ && zq < a.nproj && zr >= (int)mbeg + k * PT_ROWS - mb && zr < (int)mend - mb;
    if (T == 256 || tid < 256) dzL[k & 1][tid] = ok ? v : 0.0f;
  };
  auto put_z = [&](int k) __attribute__((always_inline)) { put_zv(k, rz); };

  float db = 0.f, dzs = 0.f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float e[RP];
  uint32_t w[RP / 2][3];
  float4 zv[RP];
  float zsv[RP];
  auto z_read = [&](int c, int i0, int n) __attribute__((always_inline)) {
    if constexpr (GF) return;
    const int buf = c & 1;
#pragma unroll
    for (int i = i0; i < i0 + n; ++i) {
      const int r = RP * go + i;
      zv[i] = *reinterpret_cast<const float4*>(&dzL[buf][r * MAXPROJ]);
      zsv[i] = dzL[buf][r * MAXPROJ + (gn & (MAXPROJ - 1))];
    }
  };
  auto put_a = [&](int s, int j, int c) __attribute__((always_inline)) {
    *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(At[c & 1]) + loff[j]) = ra[s][j];
  };
  auto g_row = [&](int i, int c, int half, int sg) __attribute__((always_inline)) {
    if constexpr (GF) {  // G itself (rows past the block's end: zero)
      if (half == 0) return;
      const int mb = ldbase(c);
      const int r = RP * go + i;
      const bool ok = r >= (int)mbeg + c * PT_ROWS - mb && r < (int)mend - mb && gcol;
      const float g = ok ? rg[sg][i] : 0.0f;
      db += g;
      e[i] = g * gsc;  // exact (a power of two)
      return;
    }
    if (half == 0) {
      const float4 z = zv[i];
      float g = z.x * pcol[0];
      g = fmaf(z.y, pcol[1], g);
      g = fmaf(z.z, pcol[2], g);
      e[i] = fmaf(z.w, pcol[3], g);
      dw2[0] = fmaf(z.x, rg[sg][i], dw2[0]);
      dw2[1] = fmaf(z.y, rg[sg][i], dw2[1]);
      dw2[2] = fmaf(z.z, rg[sg][i], dw2[2]);
      dw2[3] = fmaf(z.w, rg[sg][i], dw2[3]);
      return;
    }
    float g = e[i];
    dzs += gn < MAXPROJ ? zsv[i] : 0.0f;
    g = rg[sg][i] > 0.0f ? g * a.hscale : 0.0f;
    db += g;
    if constexpr (GOUT) {
      const int mb = ldbase(c);
      const int r = RP * go + i;
      const bool ok = r >= (int)mbeg + c * PT_ROWS - mb && r < (int)mend - mb && gcol;
      if (a.gout && ok) a.gout[(int64_t)(mb + r) * a.ldgout + gn] = g;
    }
    e[i] = g * gsc;  // exact (a power of two)
  };
  auto split_pair = [&](int j) __attribute__((always_inline)) {
    split_h2_pair(e[2 * j], e[2 * j + 1], w[j][1], w[j][2]);
    w[j][0] = h2_scale_pair(w[j][1], 2048.0f);
  };
  auto g_put = [&](int c) __attribute__((always_inline)) {
    uint16_t* gd = Gt[c & 1] + gn * PT_GP + RP * go;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if constexpr (RP == 8) *reinterpret_cast<uint4*>(gd + p * PT_GPL) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
      else *reinterpret_cast<uint2*>(gd + p * PT_GPL) = make_uint2(w[0][p], w[1][p]);
    }
  };
  // staging unit k of chunk c + 1 (refills for chunks c + 2 / c + 3); same order as the
  // split-image kernel: A pieces, dz reads, G rows, splits, G write, h loads, dz ring
  // (par: c's parity, a compile-time constant after inlining — chunk c + 1's pieces sit in set
  // (c + 1) % RING, refilled with chunk c + 1 + RING)
  auto unit = [&](int k, int c, int par) __attribute__((always_inline)) {
    constexpr int Z0 = 2 * NPA, G0 = Z0 + RP / 2, S0 = G0 + 2 * RP, P0 = S0 + RP / 2;
    const int sa = RING == 1 ? 0 : (par ^ 1);
    const int sg = RGN == 1 ? 0 : (par ^ 1);  // chunk c + 1's G rows
    if (k < Z0) {
      if (k & 1) load_a(sa, k >> 1, min(c + 1 + RING, clast));
      else put_a(sa, k >> 1, c + 1);
    } else if (k < G0) {
      z_read(c + 1, 2 * (k - Z0), 2);
    } else if (k < S0) {
      g_row((k - G0) >> 1, c + 1, (k - G0) & 1, sg);
    } else if (k < P0) {
      split_pair(k - S0);
    } else if (k == P0) {
      g_put(c + 1);
    } else if (k == P0 + 1) {
      load_g(sg, min(c + 1 + RGN, clast));
    } else if (k == P0 + 2) {
      put_z(c + 2);
      load_z(min(c + 3, clast));
    }
  };

  const int gfo = (wrow + (lane & 31)) * PT_GP + 8 * (lane >> 5);
  const int grp = lane >> 4, li = lane & 15;
  const int afo = (8 * (grp >> 1) + (li >> 2)) * PT_AP + 16 * (grp & 1) + 4 * (li & 3);
  auto afrag = [&](const uint16_t* base, int t, int p) __attribute__((always_inline)) {
    const uint16_t* q = base + p * PT_APL + t * 32;
    return __builtin_bit_cast(f16x8, cat_frag(tr_read(q), tr_read(q + 4 * PT_AP)));
  };
#define TH_FENCE __builtin_amdgcn_sched_barrier(0)
  auto compute = [&](int c, auto parc) __attribute__((always_inline)) {
    constexpr int par = decltype(parc)::value;
    const int buf = c & 1;
    f16x8 gf[3], af[2][2];  // G: hi', hi, lo; A: hi, lo
#pragma unroll
    for (int p = 0; p < 3; ++p) gf[p] = *reinterpret_cast<const f16x8*>(Gt[buf] + p * PT_GPL + gfo);
    const uint16_t* ab = At[buf] + afo;
#pragma unroll
    for (int p = 0; p < 2; ++p) af[0][p] = afrag(ab, tbase, p);
    constexpr int pg[3] = {2, 1, 0}, pa[3] = {0, 1, 0};  // G_lo·A_hi, G_hi·A_lo, G_hi'·A_hi
    static_for<KTW>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;  // this wave's t-th k-tile: tbase + t
      if constexpr (t + 1 < KTW && !(LAB & 4)) {
#pragma unroll
        for (int p = 0; p < 2; ++p) af[(t + 1) & 1][p] = afrag(ab, tbase + t + 1, p);  // (past ntl: unused)
      }
      static_for<3>([&](auto mc) __attribute__((always_inline)) {
        constexpr int m = decltype(mc)::value;
        constexpr int gap = 3 * t + m;
        TH_FENCE;
        if constexpr (!(LAB & 1)) {
          if (NW == 4 || t < ntl)  // wave-uniform
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(gf[pg[m]], af[(LAB & 4) ? 0 : (t & 1)][pa[m]], acc[t], 0, 0, 0);
        }
        TH_FENCE;
        if constexpr (!(LAB & 2)) {
          static_for<(gap + 1) * NU / NG - gap * NU / NG>([&](auto uc) __attribute__((always_inline)) {
            unit(gap * NU / NG + decltype(uc)::value, c, par);
          });
        }
      });
      TH_FENCE;
    });
    if constexpr (NU > NG) {}  // every unit is placed inside the chain (NU units over NG gaps)
    if constexpr ((LAB & 1) != 0) {
#pragma unroll
      for (int t = 0; t < KTW; ++t) acc[t][0] += (float)gf[0][0] + (float)af[0][0][0] + (float)af[1][1][1];
    }
  };
#undef TH_FENCE

  if (nch > 0) {
    // every prologue load issued before the first use of any (round 6): chunk 0's A pieces and G
    // rows, then the dz values of chunks 0..2 together — the dz ring's two LDS puts used to wait
    // one round trip each before chunk 0's loads were even issued (the TN's fixed cost on a
    // strong-scaling shard, where a block walks only ~8 chunks)
#pragma unroll
    for (int j = 0; j < NPA; ++j) load_a(0, j, 0);
    if constexpr (RING == 2) {
#pragma unroll
      for (int j = 0; j < NPA; ++j) load_a(1, j, min(1, clast));
    }
    load_g(0, 0);
    if constexpr (RGN == 2) load_g(1, min(1, clast));
    float* dzb = reinterpret_cast<float*>(&At[0][0]) + NW * 2 * 256;  // CSC: the block's dz rows
    if constexpr (CSC && !GF) {  // this block's dz[:, 0:ccols] (At is scratch until chunk 0's put)
      zm_fold = tn_csc_fold<NW>(a, mbeg, mend, reinterpret_cast<float*>(&At[0][0]) + wave * 2 * 256, dzb, lane, wave);
      __syncthreads();  // the block's dz rows written (a workgroup fence) before any wave reads them
    }
    float rz0 = 0.f, rz1 = 0.f;
    if constexpr (CSC && !GF) {  // chunks 0 and 1 from the fold's LDS rows (rows outside the block: masked)
      auto dzb_at = [&](int c) __attribute__((always_inline)) {
        const int64_t rl = ldbase(c) + zr - mbeg;
        return (rl >= 0 && rl < mend - mbeg) ? dzb[rl * MAXPROJ + zq] : 0.f;
      };
      rz0 = dzb_at(0);
      rz1 = dzb_at(min(1, clast));
    } else if constexpr (!GF) {
      rz0 = a.dz[(uint32_t)((ldbase(0) + zr) * (int)a.lddz + zqc)];
      rz1 = a.dz[(uint32_t)((ldbase(min(1, clast)) + zr) * (int)a.lddz + zqc)];
    }
    load_z(min(2, clast));
    put_zv(0, rz0);
    put_zv(1, rz1);
    scan_scale();     // (its barrier also publishes dzL)
#pragma unroll
    for (int j = 0; j < NPA; ++j) put_a(0, j, 0);
    z_read(0, 0, RP);
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      g_row(i, 0, 0, 0);
      g_row(i, 0, 1, 0);
    }
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) split_pair(j);
    g_put(0);
#pragma unroll
    for (int j = 0; j < NPA; ++j) load_a(0, j, min(RING, clast));  // set 0: chunk RING (1 or 2)
    load_g(0, min(RGN, clast));  // set 0: chunk RGN (1 or 2)
    __syncthreads();
    for (int c = 0; c < nch; c += 2) {  // unrolled by 2: the ring's set indices are static
      compute(c, std::integral_constant<int, 0>{});
      __syncthreads();
      if (c + 1 < nch) {
        compute(c + 1, std::integral_constant<int, 1>{});
        __syncthreads();
      }
    }
  }

  // ---- this block's partial dW (segment-major: dW1 = [Nr][k1] then dW2 = [Nr][k2])
  float* slab = a.slab + (int64_t)rblk * a.slab_stride;
  const int Kc = a.k1 + a.k2;
#pragma unroll
  for (int t = 0; t < KTW; ++t) {
    if (NW == 8 && t >= ntl) break;  // wave-uniform
    const int kp = (kt0 + tbase + t) * 32 + (lane & 31);
    const bool s1 = kp < a.k1;
    const bool s2 = kp >= a.ap_col2 && kp < a.ap_col2 + a.k2;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wrow + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t idx = s1 ? (int64_t)row * a.k1 + kp : (int64_t)a.Nr * a.k1 + (int64_t)row * a.k2 + (kp - a.ap_col2);
      if constexpr ((LAB & 128) != 0) {  // lab: no slab stores (one per wave keeps the chain live)
        if (row < a.Nr && (s1 || s2) && acc[t][r] == 1.2345f) slab[idx] = 0.f;
      } else {
        if (row < a.Nr && (s1 || s2)) slab[idx] = acc[t][r] * gunsc;
      }
    }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(&At[0][0]);
  constexpr int ns = 2 + MAXPROJ;
  red[(go * 128 + gn) * ns + 0] = db;
  red[(go * 128 + gn) * ns + 1] = dzs;
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) red[(go * 128 + gn) * ns + 2 + q] = dw2[q];
  __syncthreads();
  constexpr int NGO = T / 128;  // row groups of a column, combined in order
  auto comb = [&](int col, int f) __attribute__((always_inline)) {
    float v = red[col * ns + f];
#pragma unroll
    for (int o = 1; o < NGO; ++o) v += red[(o * 128 + col) * ns + f];
    return v;
  };
  if (kpart != 0) return;  // (split-K: the side sums once per row block)
  if (tid < 128 && tid < a.Nr) {
    float* side = slab + (int64_t)a.Nr * Kc;
    side[tid] = comb(tid, 0);
    for (int q = 0; q < a.nproj; ++q) side[a.Nr + q * a.Nr + tid] = comb(tid, 2 + q);
  }
  if (tid < a.nproj) slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = comb(tid, 1);
}

// ------------------------------------------------------------------ TN over a bf16 image
// bf16 storage (BASELINE configs[4]): A = a one-plane bf16 image (planes.BfImage), h bf16, G
// rounded to bf16 for the MFMA (one product), f32 accumulation.  One MFMA per k-tile per 16-row
// chunk (11 per wave at K = 336) is far too short a phase to hide a chunk's loads behind, so the
// loads run D chunks ahead in a register ring (slots indexed at compile time: the chunk loop is
// unrolled by D):
//   step c:  A(c+1) pieces -> LDS, G(c+1) formed from the ring slot and dz(c+1) -> LDS (bf16)
//            | the slot refilled with chunk c+1+D | dz(c+2) -> the LDS dz ring, its slot refilled
//            with dz(c+2+D) | the KT MFMAs of chunk c | barrier
// Geometry, the G formation, masks, side sums and slab layout are the split-image kernel's above.
// GB: g (the g form's input) and gout are bf16 rows — the bf16-storage backward keeps the hidden
// layers' input gradients in bf16 (autocast's rounding points: G and dh stored bf16).
template <bool PROJ, bool MASK, int KT, bool GOUT, int D, bool GB = false>
__global__ __launch_bounds__(256) void gemm_tn_img16_kernel(TNArgs a) {
  constexpr int NPA = 3;  // A pieces per thread per chunk (16 rows x <= 42 pieces <= 768)
  __shared__ __attribute__((aligned(16))) uint16_t Gt[2][PT_GPL];
  __shared__ __attribute__((aligned(16))) uint16_t At[2][PT_APL];
  __shared__ float dzL[2][256];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ld = a.ap_ld;
  const int pr = ld >> 3;
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);
  const int nch = mend > mbeg ? (int)((mend - mbeg + PT_ROWS - 1) / PT_ROWS) : 0;

  floatx16 acc[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  const __amdgpu_buffer_rsrc_t arsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.ap), 0, (int)(a.ap_ps * 2), 0x00020000);
  uint32_t goff[NPA], loff[NPA];
#pragma unroll
  for (int j = 0; j < NPA; ++j) {
    const int q = tid + 256 * j;
    const bool ok = q < PT_ROWS * pr;
    const int row = q / pr, c16 = q - row * pr;
    goff[j] = ok ? (uint32_t)(((int64_t)row * ld + 8 * c16) * 2) : 0u;
    loff[j] = ok ? (uint32_t)((row * PT_AP + 8 * c16) * 2)
                 : (uint32_t)(((tid & 15) * PT_AP + PT_MAXLD + 8 * ((tid >> 4) & 1)) * 2);
  }
  // G slot: columns n0 .. n0 + 4 (one vector load / store per row), rows 2·rp, 2·rp + 1 of the
  // chunk.  Few, wide memory operations per chunk keep the ring's loads countable (vmcnt <= 63).
  const int gc4 = tid & 31, rp = tid >> 5;
  const int n0 = 4 * gc4;
  const bool gcol = n0 < a.Nr;  // Nr % 4 == 0: all four columns or none
  const int n0c = gcol ? n0 : 0;
  const uint16_t* hbase = reinterpret_cast<const uint16_t*>(a.h) + n0c;
  const float* gbase = a.g + n0c;
  const uint16_t* gbase16 = reinterpret_cast<const uint16_t*>(a.g) + n0c;
  const int zr = (tid & 63) / MAXPROJ, zq = (tid & 63) % MAXPROJ;
  const int zqc = PROJ ? min(zq, a.nproj - 1) : 0;
  float pcol[4][MAXPROJ];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) pcol[j][q] = (PROJ && q < a.nproj && gcol) ? a.proj[q * a.Nr + n0 + j] : 0.0f;

  const int Mi = (int)a.M;
  auto ldbase = [&](int c) { return min((int)mbeg + c * PT_ROWS, Mi - PT_ROWS); };
  const int clast = max(nch - 1, 0);
  // the register ring (slot d: one chunk's A pieces, the slot's h / g row vectors, a dz value)
  u32x4 ra[D][NPA];
  uint2 rh[D][2];
  float4 rg[D][2];
  uint2 rgb[D][2];
  float rz[D];
  auto load_chunk = [&](int d, int c) {  // c clamped by the caller
    const int mb = ldbase(c);
#pragma unroll
    for (int j = 0; j < NPA; ++j) ra[d][j] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)goff[j], mb * ld * 2, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t row = (uint32_t)(mb + 2 * rp + i);
      if constexpr (MASK) rh[d][i] = *reinterpret_cast<const uint2*>(hbase + row * (uint32_t)a.ldh);
      if constexpr (!PROJ && GB) rgb[d][i] = *reinterpret_cast<const uint2*>(gbase16 + row * (uint32_t)a.ldg);
      else if constexpr (!PROJ) rg[d][i] = *reinterpret_cast<const float4*>(gbase + row * (uint32_t)a.ldg);
    }
  };
  auto load_z = [&](int d, int c) {
    if constexpr (PROJ) rz[d] = a.dz[(uint32_t)((ldbase(c) + zr) * (int)a.lddz + zqc)];
  };
  auto put_z = [&](int d, int k) {  // dz of chunk k into its LDS ring slot (zero outside the block's rows)
    if constexpr (PROJ) {
      const int mb = ldbase(k);
      const bool ok = tid < PT_ROWS * MAXPROJ && zq < a.nproj && zr >= (int)mbeg + k * PT_ROWS - mb && zr < (int)mend - mb;
      dzL[k & 1][tid] = ok ? rz[d] : 0.0f;
    }
  };

  float db[4] = {0.f, 0.f, 0.f, 0.f};
  float dzs[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float dw2[4][MAXPROJ];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) dw2[j][q] = 0.f;
  // chunk c's A pieces and G block (from ring slot d) into LDS buffer c & 1
  auto put_chunk = [&](int d, int c) {
    const int buf = c & 1;
#pragma unroll
    for (int j = 0; j < NPA; ++j) *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(At[buf]) + loff[j]) = ra[d][j];
    const int mb = ldbase(c);
    float gv[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 2 * rp + i;
      const bool ok = r >= (int)mbeg + c * PT_ROWS - mb && r < (int)mend - mb && gcol;
      float hv[4];
      if constexpr (MASK) {
        hv[0] = __uint_as_float(rh[d][i].x << 16);
        hv[1] = __uint_as_float(rh[d][i].x & 0xffff0000u);
        hv[2] = __uint_as_float(rh[d][i].y << 16);
        hv[3] = __uint_as_float(rh[d][i].y & 0xffff0000u);
      }
      float4 z = {0.f, 0.f, 0.f, 0.f};
      if constexpr (PROJ) {
        z = *reinterpret_cast<const float4*>(&dzL[buf][r * MAXPROJ]);
        if (gc4 == 0) {  // Σ dz: the column-group-0 threads, one row each
          dzs[0] += z.x; dzs[1] += z.y; dzs[2] += z.z; dzs[3] += z.w;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float e;
        if constexpr (PROJ) {
          e = z.x * pcol[j][0];
          e = fmaf(z.y, pcol[j][1], e);
          e = fmaf(z.z, pcol[j][2], e);
          e = fmaf(z.w, pcol[j][3], e);
          if constexpr (MASK) {
            dw2[j][0] = fmaf(z.x, hv[j], dw2[j][0]);
            dw2[j][1] = fmaf(z.y, hv[j], dw2[j][1]);
            dw2[j][2] = fmaf(z.z, hv[j], dw2[j][2]);
            dw2[j][3] = fmaf(z.w, hv[j], dw2[j][3]);
          }
        } else if constexpr (GB) {
          const uint32_t wd = j < 2 ? rgb[d][i].x : rgb[d][i].y;
          e = __uint_as_float((j & 1) ? (wd & 0xffff0000u) : (wd << 16));
        } else {
          e = j == 0 ? rg[d][i].x : j == 1 ? rg[d][i].y : j == 2 ? rg[d][i].z : rg[d][i].w;
        }
        float g = e;
        if constexpr (MASK) g = hv[j] > 0.0f ? g * a.hscale : 0.0f;
        if constexpr (!PROJ) g = ok ? g : 0.0f;
        db[j] += g;
        gv[i][j] = g;
      }
      if constexpr (GOUT && GB) {  // the rounded G the MFMA uses, as bf16 rows
        if (a.gout && ok)
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(a.gout) + (int64_t)(mb + r) * a.ldgout + n0) = make_uint2(
              __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v_t){gv[i][0], gv[i][1]}, bf16x2v_t)),
              __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v_t){gv[i][2], gv[i][3]}, bf16x2v_t)));
      } else if constexpr (GOUT) {
        if (a.gout && ok)
          *reinterpret_cast<float4*>(a.gout + (int64_t)(mb + r) * a.ldgout + n0) =
              make_float4(gv[i][0], gv[i][1], gv[i][2], gv[i][3]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)  // Gt[n][rows]: the two rows of column n0 + j as one bf16 pair
      *reinterpret_cast<uint32_t*>(Gt[buf] + (n0 + j) * PT_GP + 2 * rp) =
          __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v_t){gv[0][j], gv[1][j]}, bf16x2v_t));
  };

  const int gfo = (32 * wave + (lane & 31)) * PT_GP + 8 * (lane >> 5);
  const int grp = lane >> 4, li = lane & 15;
  const int afo = (8 * (grp >> 1) + (li >> 2)) * PT_AP + 16 * (grp & 1) + 4 * (li & 3);
  auto compute = [&](int c) {
    const int buf = c & 1;
    const bf16x8 gf = *reinterpret_cast<const bf16x8*>(Gt[buf] + gfo);
    const uint16_t* ab = At[buf] + afo;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const uint16_t* q = ab + t * 32;
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf, cat_frag(tr_read(q), tr_read(q + 4 * PT_AP)), acc[t], 0, 0, 0);
    }
  };

  if (nch > 0) {
    // prologue: ring slots d hold chunk d and dz(d); dz(0), dz(1) -> LDS; chunk 0 -> LDS
#pragma unroll
    for (int d = 0; d < D; ++d) {
      load_chunk(d, min(d, clast));
      load_z(d, min(d, clast));
    }
    put_z(0, 0);
    put_z(1, 1);
    load_z(0, min(D, clast));
    load_z(1, min(D + 1, clast));
    __syncthreads();  // dzL
    put_chunk(0, 0);
    load_chunk(0, min(D, clast));
    __syncthreads();
    for (int c0 = 0; c0 < nch; c0 += D) {
      static_for<D>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        const int c = c0 + d;
        if (c < nch) {
          constexpr int d1 = (d + 1) % D, d2 = (d + 2) % D;
          put_chunk(d1, c + 1);                 // chunk c + 1 (rows past the block: zero G)
          load_chunk(d1, min(c + 1 + D, clast));
          put_z(d2, c + 2);
          load_z(d2, min(c + 2 + D, clast));
          compute(c);
          __syncthreads();
        }
      });
    }
  }

  // ---- this block's partial dW (segment-major: dW1 = [Nr][k1] then dW2 = [Nr][k2])
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  const int Kc = a.k1 + a.k2;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int kp = t * 32 + (lane & 31);
    const bool s1 = kp < a.k1;
    const bool s2 = kp >= a.ap_col2 && kp < a.ap_col2 + a.k2;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t idx = s1 ? (int64_t)row * a.k1 + kp : (int64_t)a.Nr * a.k1 + (int64_t)row * a.k2 + (kp - a.ap_col2);
      if (row < a.Nr && (s1 || s2)) slab[idx] = acc[t][r];
    }
  }
  // side sums: the two row pairs of a column group in a wave (lanes l, l + 32) by one exchange,
  // then the four waves in order through LDS (At[0] is free after the last barrier)
  constexpr int ns = 1 + MAXPROJ;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    db[j] += __shfl_xor(db[j], 32);
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) dw2[j][q] += __shfl_xor(dw2[j][q], 32);
  }
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) dzs[q] += __shfl_xor(dzs[q], 32);
  __syncthreads();
  float* red = reinterpret_cast<float*>(&At[0][0]);  // [4 waves][128 columns][ns] + [4 waves][4] dz sums
  if (lane < 32) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[(wave * 128 + n0 + j) * ns] = db[j];
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) red[(wave * 128 + n0 + j) * ns + 1 + q] = dw2[j][q];
    }
    if (gc4 == 0) {
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) red[4 * 128 * ns + wave * MAXPROJ + q] = dzs[q];
    }
  }
  __syncthreads();
  if (tid < 128 && tid < a.Nr) {
    float* side = slab + (int64_t)a.Nr * Kc;
    const float* rr = red + tid * ns;
    side[tid] = ((rr[0] + rr[128 * ns]) + rr[2 * 128 * ns]) + rr[3 * 128 * ns];
    for (int q = 0; q < a.nproj; ++q)
      side[a.Nr + q * a.Nr + tid] = ((rr[1 + q] + rr[128 * ns + 1 + q]) + rr[2 * 128 * ns + 1 + q]) + rr[3 * 128 * ns + 1 + q];
  }
  if (PROJ && tid < a.nproj) {
    const float* rz4 = red + 4 * 128 * ns;
    slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] =
        ((rz4[tid] + rz4[MAXPROJ + tid]) + rz4[2 * MAXPROJ + tid]) + rz4[3 * MAXPROJ + tid];
  }
}

template <bool PROJ, bool MASK, int KT>
void launch_tn_img16_k(const TNArgs& a, int nblk, hipStream_t st) {
  if (a.g_bf16) {
    if (a.gout) gemm_tn_img16_kernel<PROJ, MASK, KT, true, 4, true><<<nblk, 256, 0, st>>>(a);
    else gemm_tn_img16_kernel<PROJ, MASK, KT, false, 4, true><<<nblk, 256, 0, st>>>(a);
    return;
  }
  if (a.gout) gemm_tn_img16_kernel<PROJ, MASK, KT, true, 4><<<nblk, 256, 0, st>>>(a);
  else gemm_tn_img16_kernel<PROJ, MASK, KT, false, 4><<<nblk, 256, 0, st>>>(a);
}

template <int KT>
void launch_tn_img16_kt(const TNArgs& a, int nblk, hipStream_t st) {
  const bool proj = a.dz != nullptr, mask = a.h != nullptr;
  if (proj && mask) launch_tn_img16_k<true, true, KT>(a, nblk, st);
  else if (proj) launch_tn_img16_k<true, false, KT>(a, nblk, st);
  else if (mask) launch_tn_img16_k<false, true, KT>(a, nblk, st);
  else launch_tn_img16_k<false, false, KT>(a, nblk, st);
}

template <bool PROJ, bool MASK, int KT>
void launch_tn_planes_k(const TNArgs& a, int nblk, hipStream_t st) {
  if (a.Nr <= 64) {  // K split 4 ways over 8 waves (GCN / GAT layer 1, N = 64): lab GCN shape 57.2 ->
    // 53.8 us vs the 4-wave split-K (profiles/r19_lab_gemm.txt; dW bit-identical)
    if (a.gout) gemm_tn_planes_kernel<PROJ, MASK, KT, true, 0, 4, 8><<<nblk, 512, 0, st>>>(a);
    else gemm_tn_planes_kernel<PROJ, MASK, KT, false, 0, 4, 8><<<nblk, 512, 0, st>>>(a);
    return;
  }
  if constexpr (KT <= 8) {  // narrower images at N > 64 (the SAGE-ResBN layer-0 conv over x): K split 2 ways
    if (a.gout) gemm_tn_planes_kernel<PROJ, MASK, KT, true, 0, 2, 8><<<nblk, 512, 0, st>>>(a);
    else gemm_tn_planes_kernel<PROJ, MASK, KT, false, 0, 2, 8><<<nblk, 512, 0, st>>>(a);
    return;
  }
  if (a.gout) gemm_tn_planes_kernel<PROJ, MASK, KT, true><<<nblk, 256, 0, st>>>(a);
  else gemm_tn_planes_kernel<PROJ, MASK, KT, false><<<nblk, 256, 0, st>>>(a);
}

template <int KT>
void launch_tn_planes_kt(const TNArgs& a, int nblk, hipStream_t st) {
  const bool proj = a.dz != nullptr, mask = a.h != nullptr;
  if (proj && mask) launch_tn_planes_k<true, true, KT>(a, nblk, st);
  else if (proj) launch_tn_planes_k<true, false, KT>(a, nblk, st);
  else if (mask) launch_tn_planes_k<false, true, KT>(a, nblk, st);
  else launch_tn_planes_k<false, false, KT>(a, nblk, st);
}

}  // namespace

// the bf16 image form: one-plane bf16 image (ld 256 or 336), h bf16 when given
bool tn_img16_ok(const TNArgs& a) {
  if (!a.ap || a.ap_h2 || !a.a_bf16 || (a.h && !a.h_bf16)) return false;
  // the G slot's vector accesses: 4 columns per row (8-byte h, 16-byte f32 / 8-byte bf16 g and gout rows)
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  const int gb = a.g_bf16 ? 8 : 16;
  if (a.Nr % 4 || (a.h && (a.ldh % 4 || !al(a.h, 8))) || (a.g && !a.dz && (a.ldg % 4 || !al(a.g, gb))) ||
      (a.gout && (a.ldgout % 4 || !al(a.gout, gb))))
    return false;
  if ((a.ap_ld != 256 && a.ap_ld != 336) || (reinterpret_cast<uintptr_t>(a.ap) & 15)) return false;
  if (a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 || a.ap_col2 + a.k2 > a.ap_ld) return false;
  if (a.ap_ps < a.M * (int64_t)a.ap_ld || a.ap_ps * 2 >= ((int64_t)1 << 31) || a.M < PT_ROWS) return false;
  const int64_t ldmax = std::max({a.h ? a.ldh : 0, a.g ? a.ldg : 0, a.dz ? a.lddz : 0});
  return (a.M + 32) * ldmax < ((int64_t)1 << 31);
}

void launch_tn_img16(const TNArgs& a, int nblk, hipStream_t st) {
  if (a.ap_ld == 256) launch_tn_img16_kt<8>(a, nblk, st);
  else launch_tn_img16_kt<11>(a, nblk, st);
}

// the half-pair forms: the dz form with the h mask (the SAGE hidden layer), f32 h, 336-wide image
// rows; the plain g form (no dz / h / gout: G read as is, 16-byte aligned rows) over 336- or
// 176-wide images (x's x-only image: GCN / GAT layer 1, SAGE-ResBN layer 0)
bool tn_h2_ok(const TNArgs& a) {
  if (!a.ap || !a.ap_h2 || a.a_bf16 || a.h_bf16 || a.g_bf16 || (reinterpret_cast<uintptr_t>(a.ap) & 15)) return false;
  const bool gf = !a.dz && a.g && !a.h && !a.gout;
  if (gf) {
    if ((a.ap_ld != 336 && a.ap_ld != 176) || a.ldg % 4 || (reinterpret_cast<uintptr_t>(a.g) & 15)) return false;
  } else if (!a.dz || !a.proj || !a.h || a.nproj < 1 || a.ap_ld != 336) {
    return false;
  }
  // (ABI 26) the folded CSC sum: dz form without gout, 1..2 columns inside dz's nproj
  if (a.cptr && (gf || a.gout || !a.cnbr || !a.cu || a.ccols < 1 || a.ccols > 2 || a.ccols > a.nproj ||
                 a.ldu < a.ccols || a.M * a.ldu >= ((int64_t)1 << 31)))
    return false;
  if (a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 || a.ap_col2 + a.k2 > a.ap_ld) return false;
  if (a.ap_ps < a.M * (int64_t)a.ap_ld || 2 * a.ap_ps * 2 >= ((int64_t)1 << 31) || a.M < PT_ROWS) return false;
  const int64_t ldmax = gf ? a.ldg : std::max({a.ldh, a.lddz});
  return (a.M + 32) * ldmax < ((int64_t)1 << 31);
}

// 8 waves (two per SIMD, the k-tiles split between them): lab 102.3 -> 95.2 us on the headline
// shape (profiles/r19_lab_h2.txt), the staging alone 93.4 — the kernel now runs at its stream
// ks: split-K block pairs (gemm_tn_h2_kernel KS = 2; nblk = 2 x the row blocks; the dz form)
void launch_tn_h2(const TNArgs& a, int nblk, hipStream_t st, bool ks) {
  if (!a.dz) {  // the g form
    if (a.ap_ld == 176) gemm_tn_h2_kernel<6, false, 0, 8, true><<<nblk, 512, 0, st>>>(a);
    else gemm_tn_h2_kernel<11, false, 0, 8, true><<<nblk, 512, 0, st>>>(a);
    return;
  }
  if (a.cptr) {  // (ABI 26) the CSC sum of u folded in (tn_h2_ok: no gout)
    if (ks) gemm_tn_h2_kernel<11, false, 0, 8, false, 2, true><<<nblk, 512, 0, st>>>(a);
    else gemm_tn_h2_kernel<11, false, 0, 8, false, 1, true><<<nblk, 512, 0, st>>>(a);
    return;
  }
  if (ks) {
    if (a.gout) gemm_tn_h2_kernel<11, true, 0, 8, false, 2><<<nblk, 512, 0, st>>>(a);
    else gemm_tn_h2_kernel<11, false, 0, 8, false, 2><<<nblk, 512, 0, st>>>(a);
    return;
  }
  if (a.gout) gemm_tn_h2_kernel<11, true, 0, 8><<<nblk, 512, 0, st>>>(a);
  else gemm_tn_h2_kernel<11, false, 0, 8><<<nblk, 512, 0, st>>>(a);
}

bool tn_planes_ok(const TNArgs& a) {
  if (!a.ap || a.ap_h2 || a.a_bf16 || a.h_bf16 || a.g_bf16) return false;
  if (a.ap_ld % 16 || a.ap_ld > PT_MAXLD || a.ap_ld < 32) return false;
  if (a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 || a.ap_col2 + a.k2 > a.ap_ld) return false;
  if (a.ap_ps < a.M * (int64_t)a.ap_ld || (reinterpret_cast<uintptr_t>(a.ap) & 15)) return false;
  if (3 * a.ap_ps * 2 >= ((int64_t)1 << 31) || a.M < PT_ROWS) return false;
  const int64_t ldmax = std::max({a.h ? a.ldh : 0, a.g ? a.ldg : 0, a.dz ? a.lddz : 0});
  return (a.M + 32) * ldmax < ((int64_t)1 << 31);
}

void launch_tn_planes(const TNArgs& a, int nblk, hipStream_t st) {
  const int kt = (a.ap_ld + 31) / 32;
  if (kt <= 4) launch_tn_planes_kt<4>(a, nblk, st);
  else if (kt <= 6) launch_tn_planes_kt<6>(a, nblk, st);
  else if (kt <= 8) launch_tn_planes_kt<8>(a, nblk, st);
  else launch_tn_planes_kt<11>(a, nblk, st);
}

}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_split_h2_f32(const float* x, int64_t ldx, int64_t rows, int64_t F, void* img, int64_t ld,
                                       int64_t plane_stride, int64_t col0, int64_t width, int32_t scale_exp,
                                       gnn_stream_t stream) {
  if (scale_exp < -100 || scale_exp > 100) return fail(GNN_ERR_INVALID_ARG, __func__, "scale_exp outside [-100, 100]");
  if (rows < 0 || F < 0 || ldx < F || width < F || (width & 1) || (col0 & 1) || col0 < 0 || col0 + width > ld ||
      plane_stride < rows * ld || (plane_stride & 1) || (ld & 1))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad shapes (width >= F, even width / col0 / ld / plane_stride)");
  if (rows == 0 || width == 0) return GNN_OK;
  if (!x && F > 0) return fail(GNN_ERR_INVALID_ARG, __func__, "null x");
  if (!img || (reinterpret_cast<uintptr_t>(img) & 3)) return fail(GNN_ERR_INVALID_ARG, __func__, "null or unaligned image");
  const int64_t n = rows * (width / 2);
  split_h2_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(
      x, ldx, rows, (int32_t)F, static_cast<uint16_t*>(img) + col0, ld, plane_stride, (int32_t)width,
      ldexpf(1.0f, scale_exp));
  return hip_check(hipGetLastError(), __func__);
}

extern "C" gnn_status gnn_split_planes_f32(const float* x, int64_t ldx, int64_t rows, int64_t F, void* img, int64_t ld,
                                           int64_t plane_stride, int64_t col0, int64_t width, gnn_stream_t stream) {
  if (rows < 0 || F < 0 || ldx < F || width < F || (width & 1) || (col0 & 1) || col0 < 0 || col0 + width > ld ||
      plane_stride < rows * ld || (plane_stride & 1) || (ld & 1))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad shapes (width >= F, even width / col0 / ld / plane_stride)");
  if (rows == 0 || width == 0) return GNN_OK;
  if (!x && F > 0) return fail(GNN_ERR_INVALID_ARG, __func__, "null x");
  if (!img || (reinterpret_cast<uintptr_t>(img) & 3)) return fail(GNN_ERR_INVALID_ARG, __func__, "null or unaligned image");
  const int64_t n = rows * (width / 2);
  split_planes_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(
      x, ldx, rows, (int32_t)F, static_cast<uint16_t*>(img) + col0, ld, plane_stride, (int32_t)width);
  return hip_check(hipGetLastError(), __func__);
}
