// K7a-ws — weight-stationary persistent NT GEMM for the SAGE forward (split-bf16, fp32-accurate).
//
//   C = epi([A1 | A2] · [W1 | W2]ᵀ)      A1 = agg [M, k1], A2 = h [M, k2], W = the Linear weights
//
// Shape of the hot call (SAGE preset layer 1): M = 203,769, K = 166 + 166, N = 128.  The B
// operand (3 bf16 planes × 128 × 352 pre-split = 264 KB) is far too small to be worth streaming
// through LDS per row tile — the tiled form re-stages it in each of 1,592 blocks (≈ 400 MB of
// L2→LDS per launch, more than the 270 MB A stream).  Here it is STATIONARY IN REGISTERS:
//   * one persistent 512-thread block per CU (8 waves, 2 per SIMD).  Wave w owns output columns
//     32·(w&3) .. +32 and HALF of the k-steps (w < 4: the first ceil(NKS/2), w >= 4: the rest);
//     its B fragments (≤ 11 k-steps × 3 planes × 4 VGPRs) stay in registers for the launch;
//   * the block sweeps 32-row tiles of A (t = blockIdx.x, += gridDim.x).  Each tile is loaded as
//     flat dwordx4 quads (A segments contiguous: lda == k), split into hi/mid/lo bf16 (RNE,
//     exact remainders) ONCE per element by the thread that loaded it, and written to one of two
//     static LDS buffers in the MFMA fragment layout [plane][k-step][row 32][16 k] (8-row XOR
//     swizzle of the 16-byte halves: conflict-free ds_read_b128).  Tile t+1's loads are issued
//     before tile t's MFMAs and staged between them (sched_barrier fences keep the order);
//   * the two waves of a column group sum their K-half accumulators through LDS (each keeps
//     16 of the 32 rows), then run the epilogue on their rows: bias, ReLU, counter-hash dropout
//     (bit-identical to keep_elem) and the output layer's projection z = h·Pᵀ (per-wave partial
//     sums over 32 columns, added across the 4 column groups in a fixed order).
// Two waves per SIMD hide each other's LDS / HBM / barrier latency under the MFMAs; HBM traffic
// is the algorithmic minimum: A once (270 MB), C once (104 MB).
#include "gemm_common.hpp"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

namespace gnnmp {
namespace {

constexpr int WS_ROWS = 32;            // rows per tile (the MFMA M)
constexpr int WS_KSB = 32 * 32 + 32;   // bytes per k-step block of one plane: [row 32][32 B] + 32 B pad

__device__ __forceinline__ uint32_t ws_pk(float a, float b) {  // RNE, a in the low half
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}

__device__ __forceinline__ void ws_split(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = ws_pk(a, b);
  a -= __uint_as_float(h << 16);
  b -= __uint_as_float(h & 0xffff0000u);
  m = ws_pk(a, b);
  a -= __uint_as_float(m << 16);
  b -= __uint_as_float(m & 0xffff0000u);
  l = ws_pk(a, b);
}

// The MFMA as an asm statement so its B operand (the stationary weights) can be read straight
// from the accumulator file: hipcc keeps MFMA sources in VGPRs and, with 264 registers of B,
// would copy every fragment back from AGPRs (4 v_accvgpr_read per MFMA — as many VALU
// instructions as the whole epilogue).  Hazards hipcc does not pad for an asm statement
// (cdna_hip_programming.md §5.7): the chain's first MFMA takes the literal 0 as C (no VALU write
// of the accumulator before it), chained MFMAs read C back to back (0 states), and ws_mfma_end
// pads 24 states before any other instruction touches the result.  The B registers are written
// once, by the global loads of the prologue.
template <bool FIRST>
__device__ __forceinline__ void ws_mfma(floatx16& acc, const bf16x8& x, const bf16x8& b) {
  if constexpr (FIRST) asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=v"(acc) : "v"(x), "a"(b));
  else asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "a"(b));
}
__device__ __forceinline__ void ws_mfma_end(floatx16& acc) { asm volatile("s_nop 15\n\ts_nop 7" : "+v"(acc)); }

// byte offset of bf16 element (row, kk) inside one plane of an A buffer
__device__ __forceinline__ uint32_t ws_off(int row, int kk) {
  return (uint32_t)((kk >> 4) * WS_KSB + row * 32 + ((((kk >> 3) & 1) ^ ((row >> 3) & 1)) << 4) + ((kk & 7) << 1));
}

// Flags of the fused epilogue (compile-time: the interleaved loop must stay one basic block).
constexpr int WS_BIAS = 1, WS_RELU = 2, WS_DROP = 4, WS_PROJ = 8;
constexpr int WS_KMASK = 16;  // half-pair NT: dropout from precomputed keep bits (NTArgs::kmask)

// KS = 1: 4 waves (one per SIMD), every wave holds all NKS k-steps of its columns (≤ 264 VGPRs
//         of B; 512-register waves).  KS = 2: 8 waves (two per SIMD), each holds half the
//         k-steps; the pair's partial sums meet through LDS.
// r10 ablations (layer-1 shape, fused epilogue / plain store, us): production 145 / 117, no staging
// 120 / 91, no epilogue 110, neither 78.5 (the bare MFMA loop), no MFMAs 89 / 83, L2-hot A 140 /
// 109: MFMA loop 78 + staging ~27 + fused epilogue ~30.  The split-image form below (planes)
// interleaves the staging and the epilogue into the MFMA chain.
template <int NKS, int EPI, int KS>
__global__ __launch_bounds__(256 * KS) void gemm_nt_ws_kernel(NTArgs a, const uint4* __restrict__ bimg, int ntiles,
                                                             const float* __restrict__ tail) {
  constexpr int WS_THREADS = 256 * KS;
  constexpr int PLB = NKS * WS_KSB;        // bytes per plane
  constexpr int BUF = 3 * PLB;             // bytes per A buffer
  constexpr int KH0 = (NKS + KS - 1) / KS; // k-steps of the first K part (waves 0-3)
  constexpr int KH = KH0;                  // register slots per wave (the second part has <= KH0)
  constexpr int QN = (128 * NKS + WS_THREADS - 1) / WS_THREADS;  // staged quads per thread per tile
  constexpr int RV = 16 / KS;              // accumulator rows (r-slots) a wave finishes
  // LDS: two A buffers, the C tile of the epilogue ([32 rows][128] f32: coalesced C stores and
  // the projection read it), the K-half exchange (KS 2: aliased onto the C tile when the A
  // buffers leave no room — one more barrier per tile) and the projection weights.
  constexpr int CT_BYTES = WS_ROWS * BN * 4;
  constexpr int XCH_BYTES = KS == 2 ? 2 * 4 * 8 * 64 * 4 : 0;
  constexpr bool XALIAS = KS == 2 && 2 * BUF + CT_BYTES + XCH_BYTES + MAXPROJ * (BN + 16) * 4 > 163840;
  __shared__ __attribute__((aligned(16))) char A0[BUF];
  __shared__ __attribute__((aligned(16))) char A1[BUF];
  __shared__ __attribute__((aligned(16))) char CT[CT_BYTES + (XALIAS ? 0 : XCH_BYTES)];
  constexpr int PLP = BN + 16;  // PL row pitch: the 4 q rows x 4 part chunks of a read hit distinct banks
  __shared__ __attribute__((aligned(16))) float PL[MAXPROJ * PLP];  // projection weights [q][col]
  float* const ctile = reinterpret_cast<float*>(CT);
  float* const xbase = reinterpret_cast<float*>(CT + (XALIAS ? 0 : CT_BYTES));  // [2][4 groups][8][64]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int grp = wave & 3;        // column group
  const int half = KS == 2 ? wave >> 2 : 0;  // K part (and, in the epilogue, row half)
  // kernel arguments into registers once (a per-lane select of a struct field would compile to
  // a vector load of the kernarg segment)
  const float* const pa1 = a.a1;
  const float* const pa2 = a.a2 ? a.a2 : a.a1;
  const int k1 = a.k1, k2 = a.k2;
  const int64_t M = a.M;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;

  // ---- stationary B: columns 32·grp .. +32, k-steps of this wave's half, 3 planes
  //      (bimg: [chunk][plane][2n + kh], zero for n >= Nc and k >= k_g)
  const int s0 = half ? KH0 : 0;
  const int ns = half ? NKS - KH0 : KH0;
  bf16x8 bw[KH][3];
  {
    const int slot = 2 * (32 * grp + (lane & 31)) + (lane >> 5);
#pragma unroll
    for (int s = 0; s < KH; ++s) {
      const int c = min(s0 + s, NKS - 1);  // the second half may have one k-step less: its last
#pragma unroll                              // slot is loaded but never used
      for (int p = 0; p < 3; ++p) bw[s][p] = __builtin_bit_cast(bf16x8, bimg[(c * 3 + p) * 256 + slot]);
    }
  }

  // ---- zero the pad columns of both buffers once (k in [k1 + k2, 16·NKS): the staging never
  //      writes them; B is zero there but LDS garbage could be NaN)
  {
    const int npad = NKS * 16 - k1 - k2;
    for (int i = tid; i < 2 * 3 * WS_ROWS * npad; i += WS_THREADS) {
      const int c = i % npad, rest = i / npad;
      const int row = rest % WS_ROWS, bp = rest / WS_ROWS;  // bp = buffer * 3 + plane
      const int kk = k1 + k2 + c;
      char* base = (bp / 3 == 0 ? A0 : A1) + (bp % 3) * PLB;
      *reinterpret_cast<uint16_t*>(base + ws_off(row, kk)) = 0;
    }
  }

  // ---- per-thread staging map (tile-invariant): quad i -> flat element f = 4q of segment g.
  //      Idle quads (q >= nq) stage zeros into the pad bytes of k-step 0 (never read).
  uint32_t qoff[QN];               // LDS byte offsets of the quad's two pairs (pair 2 << 16 | pair 1)
  int32_t qf[QN];                  // flat element offset inside the tile's segment
  uint32_t qseg2 = 0;              // bit i: quad i in segment 2
  const int nq1 = 8 * k1, nq = nq1 + 8 * k2;  // quads per tile (32 rows · k / 4)
#pragma unroll
  for (int i = 0; i < QN; ++i) {
    const int q = tid + WS_THREADS * i;
    const bool seg2 = q >= nq1;
    const int kg = seg2 ? k2 : k1;
    const int f = 4 * (seg2 ? q - nq1 : q);
    const int row = f / max(kg, 1), col = f - row * kg;
    const int so = seg2 ? k1 : 0;  // K concatenated: segment 2 starts at k1 (even: pairs stay in a k-step)
    const bool ok = q < nq;
    const uint32_t o0 = ok ? ws_off(row, so + col) : 1024u;
    const uint32_t o1 = ok ? (col + 2 < kg ? ws_off(row, so + col + 2) : ws_off(row + 1, so)) : 1028u;
    qoff[i] = (o1 << 16) | o0;  // PLB < 64 KB
    qf[i] = ok ? f : 0;
    qseg2 |= (ok && seg2) ? (1u << i) : 0u;
  }

  // Staging registers, two sets: the quads of tile t+G are staged from one set during tile t's
  // k-loop, and each quad's registers are refilled with tile t+3G right after (prefetch depth 2:
  // every load has two tiles of MFMAs to land).
  float4 st[2][QN];
  // quad i of tile t into set `sb`: one unconditional 16-byte load (tile starts are 16-byte
  // aligned: 32·k·4 bytes).  The last tile is read from `tail`, a zero-padded copy of its rows
  // made by ws_tail_kernel, and tiles past the end re-read it (never staged into a used
  // buffer), so the loads carry no branches: hipcc's vmcnt bookkeeping then waits for exactly
  // the quad being staged instead of draining every prefetch in flight.
  const float* const tail1 = tail;
  const float* const tail2 = tail + WS_ROWS * k1;
  // the tile's two segment bases, formed once per tile (not per quad: per-quad forms compiled
  // to a scalar branch pair per load inside the MFMA stream)
  auto tile_base = [&](int t, const float*& b1, const float*& b2) {
    const int tc = min(t, ntiles - 1);
    const bool last = tc == ntiles - 1;
    b1 = last ? tail1 : pa1 + (int64_t)tc * WS_ROWS * k1;
    b2 = last ? tail2 : pa2 + (int64_t)tc * WS_ROWS * k2;
  };
  auto load_quad_b = [&](int sb, int i, const float* b1, const float* b2) {
    const bool s2 = (qseg2 >> i) & 1u;
    // idle quads (qf = 0) re-load the tile's first quad and stage it into the never-read pad
    // bytes; no zeroing (a select on the loaded value made hipcc wait for the load right there)
    st[sb][i] = *reinterpret_cast<const float4*>((s2 ? b2 : b1) + qf[i]);
  };
  auto load_quad = [&](int sb, int i, int t) {
    const float *b1, *b2;
    tile_base(t, b1, b2);
    load_quad_b(sb, i, b1, b2);
  };
  // stage one pair (half a quad: elements 2h, 2h+1) of quad i: split + 3 plane writes
  auto stage_pair = [&](char* buf, int sb, int i, int h) {
    uint32_t hi, mi, lo;
    if (h == 0) ws_split(st[sb][i].x, st[sb][i].y, hi, mi, lo);
    else ws_split(st[sb][i].z, st[sb][i].w, hi, mi, lo);
    const uint32_t o = h == 0 ? (qoff[i] & 0xffffu) : (qoff[i] >> 16);
    *reinterpret_cast<uint32_t*>(buf + o) = hi;
    *reinterpret_cast<uint32_t*>(buf + PLB + o) = mi;
    *reinterpret_cast<uint32_t*>(buf + 2 * PLB + o) = lo;
  };
  auto stage_quad = [&](char* buf, int sb, int i) {
    stage_pair(buf, sb, i, 0);
    stage_pair(buf, sb, i, 1);
  };

  const int frow = lane & 31;
  const uint32_t foff = (uint32_t)(frow * 32 + (((lane >> 5) ^ ((frow >> 3) & 1)) << 4)) + s0 * WS_KSB;
  const int col = 32 * grp + (lane & 31);
  const bool colok = col < a.Nc;
  const int Nc = a.Nc;
  const uint32_t hstep = (uint32_t)Nc * kDropGolden;
  if constexpr ((EPI & WS_PROJ) != 0) {
    for (int i = tid; i < MAXPROJ * BN; i += WS_THREADS) {
      const int q = i / BN, c = i % BN;
      PL[q * PLP + c] = (q < a.nproj && c < Nc) ? a.proj[(int64_t)q * Nc + c] : 0.f;
    }
  }
  float* const cptr = a.c;
  const int64_t ldc = a.ldc;
  // C and z leave through buffer stores: the descriptor's range check drops rows >= M (and a
  // NULL C), so every tile issues the same store instructions on every path — with branches
  // around them hipcc's vmcnt bookkeeping had to assume skipped stores and waited for A
  // prefetches issued after the quad being staged.  (nt_ws_ok: C rows 16-byte aligned,
  // Nc % 4 == 0, both buffers < 2 GB.)
  const __amdgpu_buffer_rsrc_t crsrc =
      __builtin_amdgcn_make_buffer_rsrc(cptr, 0, cptr ? (int)(M * ldc * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t zrsrc =
      __builtin_amdgcn_make_buffer_rsrc(a.z, 0, (EPI & WS_PROJ) != 0 ? (int)(M * a.ldz * 4) : 0, 0x00020000);

  // MFMAs of this wave's K half from `cur`; the next tile's quads split into `nxt` in between
  auto kloop = [&](const char* cur, char* nxt, int sb, int tload) {
    const float *lb1, *lb2;
    tile_base(tload, lb1, lb2);
    floatx16 acc;
    constexpr int SQ0 = KH - QN > 0 ? KH - QN : 0;  // k-steps SQ0.. stage one quad each
    // one fragment set, each plane re-read for step s+1 right after its last use in step s:
    // plane 2 after MFMA 1, plane 1 after MFMA 3, plane 0 after MFMA 6 — each read has 3-5
    // MFMAs (x2 waves per SIMD) to land before its next use
    bf16x8 x[3];
    auto frag = [&](int s, int p) { return *reinterpret_cast<const bf16x8*>(cur + p * PLB + s * WS_KSB + foff); };
#pragma unroll
    for (int p = 0; p < 3; ++p) x[p] = frag(0, p);
    // Program order pinned by sched_barrier fences: between two dependent MFMAs (32 cycles) the
    // wave issues the independent work of one slot — the next step's fragment reads, half a
    // staged quad (split + 3 plane writes), the refill load — so it hides under the MFMA chain.
#define WS_FENCE __builtin_amdgcn_sched_barrier(0)
#pragma unroll
    for (int s = 0; s < KH; ++s) {
      const int sn = s + 1 < KH ? s + 1 : s;
      const bool stg = s >= SQ0 && s - SQ0 < QN;  // compile-time (unrolled)
      const int qi = s - SQ0;
      const bool mm = KS == 1 || NKS % 2 == 0 || s < ns;  // odd NKS, KS 2: the
      if (mm) {                                                               // second part is 1 shorter
        if (s == 0) ws_mfma<true>(acc, x[2], bw[s][0]);  // small terms first
        else ws_mfma<false>(acc, x[2], bw[s][0]);
      }
      WS_FENCE;
      if (s + 1 < KH) x[2] = frag(sn, 2);
      if (stg) stage_pair(nxt, sb, qi, 0);
      WS_FENCE;
      if (mm) ws_mfma<false>(acc, x[1], bw[s][1]);
      WS_FENCE;
      if (stg) stage_pair(nxt, sb, qi, 1);
      WS_FENCE;
      if (mm) ws_mfma<false>(acc, x[1], bw[s][0]);
      WS_FENCE;
      if (s + 1 < KH) x[1] = frag(sn, 1);
      if (stg) load_quad_b(sb, qi, lb1, lb2);
      WS_FENCE;
      if (mm) {
        ws_mfma<false>(acc, x[0], bw[s][2]);
        ws_mfma<false>(acc, x[0], bw[s][1]);
        ws_mfma<false>(acc, x[0], bw[s][0]);
      }
      WS_FENCE;
      if (s + 1 < KH) x[0] = frag(sn, 0);
      WS_FENCE;
    }
#undef WS_FENCE
    if constexpr (KH < QN) {
#pragma unroll
      for (int i = KH; i < QN; ++i) {
        stage_quad(nxt, sb, i);
        load_quad_b(sb, i, lb1, lb2);
      }
    }
    ws_mfma_end(acc);
    return acc;
  };

  // K-half exchange of tile t.  acc holds this wave's K-half partial sums; the wave keeps
  // r-slots [8·half, 8·half + 8) (rows 16·half .. +16) and sends the other 8 to its partner.
  auto exchange_send = [&](const floatx16& acc) {
    if constexpr (KS == 2) {
      float* xo = xbase + ((half * 4 + grp) * 8) * 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) xo[j * 64 + lane] = acc[(1 - half) * 8 + j];
    }
  };
  auto exchange_recv = [&](const floatx16& acc, float (&v)[RV]) {
    if constexpr (KS == 2) {
      const float* xi = xbase + (((1 - half) * 4 + grp) * 8) * 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float o = xi[j * 64 + lane];
        const float m = acc[half * 8 + j];
        v[j] = half ? o + m : m + o;  // K-half 0 + K-half 1, same order on both waves
      }
    } else {
#pragma unroll
      for (int j = 0; j < RV; ++j) v[j] = acc[j];
    }
  };
  // E1: this wave's rows of tile t -> bias, ReLU, dropout (element row·Nc + col, bit-identical to
  // keep_elem) -> the LDS C tile.
  // bias of this lane's column, loaded once: a global load in the epilogue made hipcc wait
  // vmcnt(0) there, i.e. for every A prefetch in flight, once per tile
  float bv = 0.f;
  if constexpr ((EPI & WS_BIAS) != 0) bv = colok ? a.bias[col] : 0.f;
  auto epi_tile = [&](const float (&v)[RV], int t) {
    const int64_t rbase = (int64_t)t * WS_ROWS + 4 * (lane >> 5);
    const uint32_t h0 = ((uint32_t)rbase * (uint32_t)Nc + (uint32_t)col) * kDropGolden + (uint32_t)seed;
#pragma unroll
    for (int j = 0; j < RV; ++j) {
      const int r = half * RV + j;
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      float x = v[j] + bv;
      if constexpr ((EPI & WS_RELU) != 0) x = fmaxf(x, 0.f);
      if constexpr ((EPI & WS_DROP) != 0)
        x = keep_premixed(h0 + (uint32_t)(rl - 4 * (lane >> 5)) * hstep, seed, a.keep_thresh) ? x * a.drop_scale : 0.f;
      ctile[rl * BN + col] = colok ? x : 0.f;
    }
  };
  // E2 (after a barrier): coalesced C stores of tile t and the projection z = h·Pᵀ from the tile:
  // thread -> (row, q, part) computes a 128/NP-long dot product; the NP parts (adjacent lanes)
  // are summed in a fixed order.
  auto epi_store = [&](int t) {
    const int64_t r0 = (int64_t)t * WS_ROWS;
    {
      constexpr int NQ4 = WS_ROWS * BN / 4 / WS_THREADS;  // float4 chunks per thread
#pragma unroll
      for (int i = 0; i < NQ4; ++i) {
        const int u = tid + WS_THREADS * i;
        const int rl = u / (BN / 4), c4 = (u % (BN / 4)) * 4;
        const float4 x = *reinterpret_cast<const float4*>(ctile + rl * BN + c4);
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 xv = {__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z), __float_as_uint(x.w)};
        // columns >= Nc: an offset past the range (dropped); rows >= M fall past it by themselves
        const uint32_t off = c4 < Nc ? (uint32_t)(((r0 + rl) * ldc + c4) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(xv, crsrc, (int)off, 0, 0);
      }
    }
    if constexpr ((EPI & WS_PROJ) != 0) {
      // part p takes the float4 chunks j ≡ p (mod NP): a 16-lane read group touches 4 q rows ×
      // 4 adjacent chunks = 64 distinct banks
      constexpr int NP = WS_THREADS / (WS_ROWS * MAXPROJ);  // parts per dot product: 2 or 4
      const int part = tid % NP, q = (tid / NP) % MAXPROJ, rl = tid / (NP * MAXPROJ);
      const float4* hrow = reinterpret_cast<const float4*>(ctile + rl * BN);
      const float4* prow = reinterpret_cast<const float4*>(PL + q * PLP);
      float acc0 = 0.f, acc1 = 0.f;
#pragma unroll 2
      for (int j = part; j < BN / 4; j += 2 * NP) {  // 2 trips unrolled: bounded LDS loads in flight
        const float4 h0_ = hrow[j], p0 = prow[j];
        const float4 h1_ = hrow[j + NP], p1 = prow[j + NP];
        acc0 = fmaf(h0_.x, p0.x, acc0); acc0 = fmaf(h0_.y, p0.y, acc0);
        acc0 = fmaf(h0_.z, p0.z, acc0); acc0 = fmaf(h0_.w, p0.w, acc0);
        acc1 = fmaf(h1_.x, p1.x, acc1); acc1 = fmaf(h1_.y, p1.y, acc1);
        acc1 = fmaf(h1_.z, p1.z, acc1); acc1 = fmaf(h1_.w, p1.w, acc1);
      }
      float zsum = acc0 + acc1;
      zsum += __shfl_xor(zsum, 1);
      if constexpr (NP == 4) zsum += __shfl_xor(zsum, 2);
      const int64_t row = r0 + rl;
      const uint32_t zoff = (part == 0 && q < a.nproj) ? (uint32_t)((row * a.ldz + q) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(zsum), zrsrc, (int)zoff, 0, 0);
    }
  };

  // Per tile:  kloop(t) [stages t+1 from st] | loads(t+2) into st | exchange send | BARRIER 1 |
  //            exchange recv [| BARRIER 1b when the exchange aliases the C tile] | E1: C tile |
  //            BARRIER 2 | E2: C stores + projection.
  // Tile t+2's loads are issued before tile t's C stores, so the staging waits of kloop(t+1)
  // (in-order vmcnt) never wait for those stores.  Barrier 1 publishes A(t+1) and the exchange
  // and retires every read of A(t) and of the C tile of t-1; barrier 2 publishes the C tile.
  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;
#pragma unroll
  for (int i = 0; i < QN; ++i) load_quad(0, i, t);
#pragma unroll
  for (int i = 0; i < QN; ++i) stage_quad(A0, 0, i);
  // the steady state's issue order (set 1 quads 0..QN-1, then set 0): the first trip's staging
  // waits are then the loop's own (one vmcnt per quad, counted from the same order)
#pragma unroll
  for (int i = 0; i < QN; ++i) load_quad(1, i, t + G);      // tile t + G: staged during tile t
#pragma unroll
  for (int i = 0; i < QN; ++i) load_quad(0, i, t + 2 * G);  // tile t + 2G: staged during tile t + G
  __syncthreads();
  float v[RV];
  auto finish = [&](const floatx16& acc) {
    exchange_send(acc);
    __syncthreads();
    exchange_recv(acc, v);
    if constexpr (XALIAS) __syncthreads();
    epi_tile(v, t);
    __syncthreads();
    epi_store(t);
  };
  // two tiles per trip: static A buffers (A0 -> A1 -> A0) and register sets (1, 0), so the
  // compiler sees staging writes and fragment reads as disjoint.  Past the end the staging
  // rewrites the spare buffer with stale quads (never read) and load_quad loads nothing.
  while (true) {
    finish(kloop(A0, A1, 1, t + 3 * G));  // stages t + G from set 1, refills it with t + 3G
    t += G;
    if (t >= ntiles) break;
    finish(kloop(A1, A0, 0, t + 3 * G));  // stages t + G from set 0
    t += G;
    if (t >= ntiles) break;
  }
}


// ---------------------------------------------------------------- the split-image form (K7a-p)
// A read from a split image (NTArgs::ap, gemm_planes.hip): every (plane, k-step) block of a
// tile — [row 32][16 k] bf16 in the buffer layout above, 1 KB — is ONE 16-byte buffer load per
// lane (lane l: row l/2, k-half (l & 1) ^ bit 3 of the row, i.e. its swizzled position 16·l)
// and one ds_write_b128: no split, no tail copy (rows past M read zeros or the next plane's rows;
// their C rows are dropped by the store range check).  4 waves (one per SIMD), each all 21
// k-steps of its 32 columns (252 AGPRs of B).
//
// Software-pipelined epilogue: tile t's MFMA chain (126 per wave) carries, one slot after each
// MFMA (sched_barrier fences pin the order, so each slot issues in an MFMA's shadow):
//   slots  0..47  E1 of the previous tile t': bias, ReLU, counter-hash dropout -> LDS C tile
//   slots 48..59  staging of tile t+G (6 pieces: ds_write_b128, then the refill load of t+2G)
//   -- barrier (every wave's E1 in the C tile) --
//   slots 60..84  E2 of t': coalesced C stores from the C tile, projection z = h·Pᵀ (NE2 = 25)
//   slots 86..105 staging, the other 10 pieces
//   -- barrier at the end of the tile (A(t+G) published, C tile reads retired) --
// The last tile's epilogue runs after the loop.  Accumulators alternate between two register
// sets (two tiles per loop trip: static roles).
// LAB (timing ablations, csrc/lab/lab_nt.hip only; the library instantiates 0): bit 1 no MFMAs,
// bit 2 no epilogue slots, bit 4 no staging slots, bit 8 no mid-tile barrier.
template <int NKS, int EPI, int LAB = 0>
__global__ __launch_bounds__(256) void gemm_nt_planes_kernel(NTArgs a, const uint4* __restrict__ bimg, int ntiles) {
  constexpr int PLB = NKS * WS_KSB;  // bytes per plane of an A buffer
  constexpr int BUF = 3 * PLB;
  constexpr int QP = (3 * NKS + 3) / 4;  // 1 KB blocks per wave per tile (NKS 21: 63 real + 1 repeat)
  // slot schedule of a tile's chain (6·NKS MFMA slots; the rest run after the chain):
  //   E1 [0, 48) | staging of QA pieces [48, SB] | barrier | E2 [60, 60 + NE2) | staging of QB
  //   pieces [86, NSLOT)
  constexpr int QA = QP < 6 ? QP : 6, QB = QP - QA;
  constexpr int SB = 48 + 2 * QA - 1;  // the mid-tile barrier follows this slot
  constexpr int NSLOT = 86 + 2 * QB;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) char A0[BUF];
  __shared__ __attribute__((aligned(16))) char A1[BUF];
  __shared__ __attribute__((aligned(16))) float CT[WS_ROWS * BN];
  constexpr int PLP = BN + 16;  // PL row pitch: the 4 q rows x 4 part chunks of a read hit distinct banks
  __shared__ __attribute__((aligned(16))) float PL[MAXPROJ * PLP];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t M = a.M;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;

  // ---- stationary B: columns 32·wave .. +32, all k-steps, 3 planes
  bf16x8 bw[NKS][3];
  {
    const int slot = 2 * (32 * wave + (lane & 31)) + (lane >> 5);
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
      for (int p = 0; p < 3; ++p) bw[s][p] = __builtin_bit_cast(bf16x8, bimg[(s * 3 + p) * 256 + slot]);
  }

  // ---- staging: block b = wave + 4i of a tile, this lane's piece at pvoff
  const int ld = a.ap_ld;
  const int prow = lane >> 1;
  const int pvoff = (prow * ld + 8 * ((lane & 1) ^ ((prow >> 3) & 1))) * 2;
  const __amdgpu_buffer_rsrc_t prsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.ap), 0, (int)(3 * a.ap_ps * 2), 0x00020000);
  u32x4 st[QP];
  auto pblk = [&](int i) { return min(wave + 4 * i, 3 * NKS - 1); };
  auto load_piece = [&](int i, int t) {
    const int b = pblk(i), p = b / NKS, s = b - p * NKS;
    const int tc = min(t, ntiles - 1);
    st[i] = __builtin_amdgcn_raw_buffer_load_b128(prsrc, pvoff, (int)((p * a.ap_ps + 16 * s) * 2) + tc * WS_ROWS * ld * 2, 0);
  };
  auto put_piece = [&](char* buf, int i) {
    const int b = pblk(i), p = b / NKS, s = b - p * NKS;
    *reinterpret_cast<u32x4*>(buf + p * PLB + s * WS_KSB + 16 * lane) = st[i];
  };

  const int frow = lane & 31;
  const uint32_t foff = (uint32_t)(frow * 32 + (((lane >> 5) ^ ((frow >> 3) & 1)) << 4));
  const int col = 32 * wave + (lane & 31);
  const int Nc = a.Nc;
  const bool colok = col < Nc;
  const uint32_t hstep = (uint32_t)Nc * kDropGolden;
  if constexpr ((EPI & WS_PROJ) != 0) {
    for (int i = tid; i < MAXPROJ * BN; i += 256) {
      const int q = i / BN, c = i % BN;
      PL[q * PLP + c] = (q < a.nproj && c < Nc) ? a.proj[(int64_t)q * Nc + c] : 0.f;
    }
  }
  float bv = 0.f;
  if constexpr ((EPI & WS_BIAS) != 0) bv = colok ? a.bias[col] : 0.f;
  float* const cptr = a.c;
  const int64_t ldc = a.ldc;
  const __amdgpu_buffer_rsrc_t crsrc =
      __builtin_amdgcn_make_buffer_rsrc(cptr, 0, cptr ? (int)(M * ldc * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t zrsrc =
      __builtin_amdgcn_make_buffer_rsrc(a.z, 0, (EPI & WS_PROJ) != 0 ? (int)(M * a.ldz * 4) : 0, 0x00020000);

  // ---- epilogue pieces of a finished tile tp (tp < 0: none yet; its stores are dropped)
  float xv[16];
  auto e1 = [&](const floatx16& acc, int j, int part, int tp) {
    const int rl = (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
    if (part == 0) {
      float x = acc[j] + bv;
      if constexpr ((EPI & WS_RELU) != 0) x = fmaxf(x, 0.f);
      xv[j] = x;
    } else if (part == 1) {
      if constexpr ((EPI & WS_DROP) != 0) {  // == keep_elem(seed, row·Nc + col), bit for bit
        const uint32_t h0 = ((uint32_t)(tp * WS_ROWS + 4 * (lane >> 5)) * (uint32_t)Nc + (uint32_t)col) * kDropGolden +
                            (uint32_t)seed;
        xv[j] = keep_premixed(h0 + (uint32_t)(rl - 4 * (lane >> 5)) * hstep, seed, a.keep_thresh) ? xv[j] * a.drop_scale
                                                                                                  : 0.f;
      }
    } else {
      CT[rl * BN + col] = colok ? xv[j] : 0.f;
    }
  };
  float4 cv[4];
  float4 ph[2][4];  // projection: two trips of (h_j, p_j, h_j+NP, p_j+NP) in flight
  float pacc0 = 0.f, pacc1 = 0.f;
  constexpr int NP = 2;  // parts per projection dot product (256 threads / (32 rows · 4 q))
  const int ppart = tid % NP, pq = (tid / NP) % MAXPROJ, prl = tid / (NP * MAXPROJ);
  auto c_read = [&](int i) {
    const int u = tid + 256 * i;
    cv[i] = *reinterpret_cast<const float4*>(CT + (u / (BN / 4)) * BN + (u % (BN / 4)) * 4);
  };
  auto c_store = [&](int i, int tp) {
    const int u = tid + 256 * i;
    const int rl = u / (BN / 4), c4 = (u % (BN / 4)) * 4;
    const u32x4 xv4 = {__float_as_uint(cv[i].x), __float_as_uint(cv[i].y), __float_as_uint(cv[i].z),
                       __float_as_uint(cv[i].w)};
    // columns >= Nc and no tile: an offset past the range (dropped); rows >= M fall past it by themselves
    const uint32_t off = (c4 < Nc && tp >= 0) ? (uint32_t)((((int64_t)tp * WS_ROWS + rl) * ldc + c4) * 4) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b128(xv4, crsrc, (int)off, 0, 0);
  };
  auto p_read = [&](int tt) {  // chunks j = part + 4·tt and j + NP of row prl / projection row pq
    const float4* hrow = reinterpret_cast<const float4*>(CT + prl * BN);
    const float4* prw = reinterpret_cast<const float4*>(PL + pq * PLP);
    const int j = ppart + 2 * NP * tt;
    ph[tt & 1][0] = hrow[j];
    ph[tt & 1][1] = prw[j];
    ph[tt & 1][2] = hrow[j + NP];
    ph[tt & 1][3] = prw[j + NP];
  };
  auto p_fma = [&](int tt) {
    const float4 h0_ = ph[tt & 1][0], p0 = ph[tt & 1][1], h1_ = ph[tt & 1][2], p1 = ph[tt & 1][3];
    pacc0 = fmaf(h0_.x, p0.x, pacc0); pacc0 = fmaf(h0_.y, p0.y, pacc0);
    pacc0 = fmaf(h0_.z, p0.z, pacc0); pacc0 = fmaf(h0_.w, p0.w, pacc0);
    pacc1 = fmaf(h1_.x, p1.x, pacc1); pacc1 = fmaf(h1_.y, p1.y, pacc1);
    pacc1 = fmaf(h1_.z, p1.z, pacc1); pacc1 = fmaf(h1_.w, p1.w, pacc1);
  };
  auto p_done = [&](int tp) {
    float zsum = pacc0 + pacc1;
    zsum += __shfl_xor(zsum, 1);
    pacc0 = pacc1 = 0.f;
    const int64_t row = (int64_t)tp * WS_ROWS + prl;
    const uint32_t zoff = (ppart == 0 && pq < a.nproj && tp >= 0) ? (uint32_t)((row * a.ldz + pq) * 4) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(zsum), zrsrc, (int)zoff, 0, 0);
  };
  constexpr int PTRIPS = BN / 4 / (2 * NP);  // 8
  // E2 slot q (0..24): C reads 0-3, C stores 4-7, then the projection R0 R1 F0 R2 F1 ... R7 F6
  // F7 done (trip tt's reads two slots ahead of its FMAs)
  constexpr int NE2 = 8 + 2 * PTRIPS + 1;
  auto e2 = [&](int q, int tp) {
    if (q < 4) c_read(q);
    else if (q < 8) c_store(q - 4, tp);
    else if constexpr ((EPI & WS_PROJ) != 0) {
      const int k = q - 8;  // 0 .. 2·PTRIPS
      if (k == 0) p_read(0);
      else if (k < 2 * PTRIPS - 1) {  // 1 .. 14: R(k+1)/2 on odd k, F(k/2 - 1) on even k
        if (k & 1) p_read((k + 1) / 2);
        else p_fma(k / 2 - 1);
      } else if (k == 2 * PTRIPS - 1) {
        p_fma(PTRIPS - 1);
      } else if (k == 2 * PTRIPS) {
        p_done(tp);
      }
    }
  };

  // one slot of tile t's chain: staging of tile t+G into nxt, epilogue of tile tp from accp
  auto slot = [&](int k, char* nxt, const floatx16& accp, int tp, int t) {
    if (k < 48) {
      if constexpr (!(LAB & 2)) e1(accp, k / 3, k % 3, tp);
    } else if (k <= SB || (k >= 86 && k < NSLOT)) {
      if constexpr (!(LAB & 4)) {
        const int i = k <= SB ? (k - 48) / 2 : QA + (k - 86) / 2;
        if (k & 1) load_piece(i, t + 2 * (int)gridDim.x);
        else put_piece(nxt, i);
      }
    } else if (k < 60 + NE2) {
      if constexpr (!(LAB & 2)) e2(k - 60, tp);
    }
  };
#define NTP_FENCE __builtin_amdgcn_sched_barrier(0)
  auto kloop = [&](const char* cur, char* nxt, floatx16& acc, const floatx16& accp, int t, int tp) {
    // fragments: plane 2 re-read for step s+1 after its last use (MFMA 0), plane 1 after MFMA 2,
    // plane 0 after MFMA 5 (the products run small terms first)
    bf16x8 x[3];
    auto frag = [&](int s, int p) { return *reinterpret_cast<const bf16x8*>(cur + p * PLB + s * WS_KSB + foff); };
#pragma unroll
    for (int p = 0; p < 3; ++p) x[p] = frag(0, p);
    constexpr int fa[6] = {2, 1, 1, 0, 0, 0}, fb[6] = {0, 1, 0, 2, 1, 0};
    // (static_for: a #pragma unroll of this 126-slot body was refused, leaving bw / st indexed
    // dynamically, i.e. in scratch)
    static_for<NKS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      static_for<6>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        NTP_FENCE;
        if constexpr (!(LAB & 1)) {
          if constexpr (s == 0 && m == 0) ws_mfma<true>(acc, x[fa[m]], bw[s][fb[m]]);
          else ws_mfma<false>(acc, x[fa[m]], bw[s][fb[m]]);
        }
        NTP_FENCE;
        if constexpr (s + 1 < NKS) {
          if constexpr (m == 0) x[2] = frag(s + 1, 2);
          if constexpr (m == 2) x[1] = frag(s + 1, 1);
          if constexpr (m == 5) x[0] = frag(s + 1, 0);
        }
        slot(6 * s + m, nxt, accp, tp, t);
        if constexpr (6 * s + m == SB && !(LAB & 8)) __syncthreads();  // every wave's E1 is in the C tile
      });
    });
    NTP_FENCE;
    static_for<(NSLOT > 6 * NKS ? NSLOT - 6 * NKS : 0)>([&](auto kc) {  // short chains: the slots past it
      constexpr int k = 6 * NKS + decltype(kc)::value;
      slot(k, nxt, accp, tp, t);
      if constexpr (k == SB && !(LAB & 8)) __syncthreads();
    });
    if constexpr ((LAB & 1) != 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = x[0][r & 7];
    }
    ws_mfma_end(acc);
  };
#undef NTP_FENCE
  auto finish = [&](const floatx16& acc, int tp) {  // the last tile's epilogue, not interleaved
#pragma unroll
    for (int k = 0; k < 48; ++k) e1(acc, k / 3, k % 3, tp);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NE2; ++q) e2(q, tp);
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;
  // prologue: tile t staged into A0, tile t+G loaded
#pragma unroll
  for (int i = 0; i < QP; ++i) load_piece(i, t);
#pragma unroll
  for (int i = 0; i < QP; ++i) put_piece(A0, i);
#pragma unroll
  for (int i = 0; i < QP; ++i) load_piece(i, t + G);
  floatx16 accA, accB;
#pragma unroll
  for (int r = 0; r < 16; ++r) accA[r] = accB[r] = 0.f;
  __syncthreads();
  int tp = -1;
  while (true) {
    kloop(A0, A1, accA, accB, t, tp);  // stages t+G into A1; epilogue of tp from accB
    __syncthreads();
    tp = t;
    t += G;
    if (t >= ntiles) {
      finish(accA, tp);
      break;
    }
    kloop(A1, A0, accB, accA, t, tp);
    __syncthreads();
    tp = t;
    t += G;
    if (t >= ntiles) {
      finish(accB, tp);
      break;
    }
  }
}

// ---------------------------------------------------------------- the half-pair form (K7a-h)
// A read from a HALF-PAIR image (gemm_planes.hip, gnn_split_h2_f32): two f16 planes per f32
// value v, pre-scaled per image by 2^ap_exp so the image's largest |u| sits in [2^13, 2^14):
//     u = v · 2^ap_exp,   hi = RNE_f16(u),   lo = RNE_f16((u - hi) · 2^11)
// (the remainder u - hi is exact in f32; u = hi + 2^-11 lo to 2^-22 |u| while hi and the scaled
// remainder are f16 normals, |u| >= 2^-13 — every value within 2^-26 of the image's largest,
// whatever the input's magnitude; below f16's normal floor only an absolute 2^-36 would remain,
// which is why the image is pre-scaled rather than stored as is).  B, from the Linear weights,
// each output column scaled by the power of two 2^-e_n that brings its largest weight into
// [8, 16), is held as THREE planes: hi' = 2^11·hi, hi, lo (hi' < 2^15 fits f16).  Three f16
// products per k-step into ONE accumulator (the split-bf16 form runs six):
//     acc += A_hi · B_hi' + A_hi · B_lo + A_lo · B_hi   (= 2^(11 + ap_exp) · A·B, up to 2^-22 relative)
//     C    = acc · 2^(e_n - 11 - ap_exp)                 (colscale: powers of two, exact)
// The dropped A_lo·B_lo term is 2^-22 relative: products good to ~2^-21 (fp32 rounds at 2^-24;
// the parity bar is 1e-5), on v_mfma_f32_32x32x16_f16 (the bf16 rate).  A moves 4 B per element
// (the split-bf16 image's 6) and the MFMA chain halves.
// Geometry and software pipeline as the split-image kernel (one 256-thread block per CU, wave w
// owns columns 32w .. +32 with B stationary in AGPRs: NKS x 3 x 4 = 252 for NKS 21), 32-row tiles
// t = blockIdx.x, += gridDim.x, two A buffers.  Slot schedule: the tile's 3·NKS MFMAs carry the
// previous tile's E1 (bias, ReLU, dropout -> LDS C tile), the staging of tile t+G, a barrier, E2
// (C stores, projection) and the rest of the staging, spread evenly (several actions per MFMA gap).
// LAB (csrc/lab only; the library instantiates 0): bit 1 no MFMAs, 2 no epilogue, 4 no staging.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int FIRST>
__device__ __forceinline__ void h2_mfma(floatx16& acc, const f16x8& x, const f16x8& b) {
  if constexpr (FIRST) asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=v"(acc) : "v"(x), "a"(b));
  else asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "a"(b));
}
__device__ __forceinline__ void h2_mfma_end(floatx16& a1) { asm volatile("s_nop 15\n\ts_nop 7" : "+v"(a1)); }

namespace h2s {
enum : int { E1 = 1, E2 = 2, SP = 3, SL = 4, BAR = 5 };
constexpr int MAXA = 200;
struct Sched {
  int kind[MAXA], idx[MAXA];
  int first[MAXA];  // first action of slot k; slot k runs actions [first[k], first[k + 1])
  int n;
};
// actions: E1 (48: element j = i/3, part i%3) interleaved with the first staging pieces, the
// barrier, E2 (ne2) interleaved with the rest; spread over nslot MFMA gaps
constexpr Sched make(int QP, int ne2, int nslot) {
  Sched s{};
  int n = 0;
  const int qa = QP / 2;  // staging pieces before the barrier
  for (int e = 0, q = 0; e < 48; ++e) {
    s.kind[n] = E1; s.idx[n++] = e;
    if (q < qa && (e + 1) * qa / 48 > q) {
      s.kind[n] = SP; s.idx[n++] = q;
      s.kind[n] = SL; s.idx[n++] = q;
      ++q;
    }
  }
  s.kind[n] = BAR; s.idx[n++] = 0;
  for (int e = 0, q = qa; e < ne2; ++e) {
    s.kind[n] = E2; s.idx[n++] = e;
    if (q < QP && qa + (e + 1) * (QP - qa) / ne2 > q) {
      s.kind[n] = SP; s.idx[n++] = q;
      s.kind[n] = SL; s.idx[n++] = q;
      ++q;
    }
  }
  s.n = n;
  for (int k = 0; k <= nslot; ++k) s.first[k] = k * n / nslot;
  return s;
}
}  // namespace h2s

template <int NKS, int EPI, int LAB = 0>
__global__ __launch_bounds__(256) void gemm_nt_h2_kernel(NTArgs a, const uint4* __restrict__ bimg,
                                                         const float* __restrict__ colscale, int ntiles) {
  constexpr int PLB = NKS * WS_KSB;  // bytes per plane of an A buffer
  constexpr int BUF = 2 * PLB;
  constexpr int QP = (2 * NKS + 3) / 4;  // 1 KB blocks per wave per tile (NKS 21: 42 -> 11, one repeat)
  constexpr int NSL = 3 * NKS;           // MFMA gaps per tile
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) char A0[BUF];
  __shared__ __attribute__((aligned(16))) char A1[BUF];
  __shared__ __attribute__((aligned(16))) float CT[WS_ROWS * BN];
  constexpr int PLP = BN + 16;
  __shared__ __attribute__((aligned(16))) float PL[MAXPROJ * PLP];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t M = a.M;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;

  f16x8 bw[NKS][3];  // hi' = 2^11 hi, hi, lo
  {
    const int slot = 2 * (32 * wave + (lane & 31)) + (lane >> 5);
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
      for (int p = 0; p < 3; ++p) bw[s][p] = __builtin_bit_cast(f16x8, bimg[(s * 3 + p) * 256 + slot]);
  }

  const int ld = a.ap_ld;
  const int prow = lane >> 1;
  const int pvoff = (prow * ld + 8 * ((lane & 1) ^ ((prow >> 3) & 1))) * 2;
  const __amdgpu_buffer_rsrc_t prsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.ap), 0, (int)(2 * a.ap_ps * 2), 0x00020000);
  u32x4 st[QP];
  auto pblk = [&](int i) __attribute__((always_inline)) { return min(wave + 4 * i, 2 * NKS - 1); };
  auto load_piece = [&](int i, int t) __attribute__((always_inline)) {
    const int b = pblk(i), p = b / NKS, s = b - p * NKS;
    const int tc = min(t, ntiles - 1);
    st[i] = __builtin_amdgcn_raw_buffer_load_b128(prsrc, pvoff, (int)((p * a.ap_ps + 16 * s) * 2) + tc * WS_ROWS * ld * 2, 0);
  };
  auto put_piece = [&](char* buf, int i) __attribute__((always_inline)) {
    const int b = pblk(i), p = b / NKS, s = b - p * NKS;
    *reinterpret_cast<u32x4*>(buf + p * PLB + s * WS_KSB + 16 * lane) = st[i];
  };

  const int frow = lane & 31;
  const uint32_t foff = (uint32_t)(frow * 32 + (((lane >> 5) ^ ((frow >> 3) & 1)) << 4));
  const int col = 32 * wave + (lane & 31);
  const int Nc = a.Nc;
  const bool colok = col < Nc;
  const uint32_t hstep = (uint32_t)Nc * kDropGolden;
  if constexpr ((EPI & WS_PROJ) != 0) {
    for (int i = tid; i < MAXPROJ * BN; i += 256) {
      const int q = i / BN, c = i % BN;
      PL[q * PLP + c] = (q < a.nproj && c < Nc) ? a.proj[(int64_t)q * Nc + c] : 0.f;
    }
  }
  float bv = 0.f;
  if constexpr ((EPI & WS_BIAS) != 0) bv = colok ? a.bias[col] : 0.f;
  const float cs = colok ? colscale[col] : 0.f;  // 2^(e_n - 11)
  float* const cptr = a.c;
  const int64_t ldc = a.ldc;
  const __amdgpu_buffer_rsrc_t crsrc =
      __builtin_amdgcn_make_buffer_rsrc(cptr, 0, cptr ? (int)(M * ldc * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t zrsrc =
      __builtin_amdgcn_make_buffer_rsrc(a.z, 0, (EPI & WS_PROJ) != 0 ? (int)(M * a.ldz * 4) : 0, 0x00020000);

  float xv[16];
  uint32_t mk[2] = {0u, 0u};  // keep-bit words: the tile being computed (loaded) / the tile in E1 (used)
  uint32_t mku = 0u;
  auto load_mk = [&](uint32_t& m, int t) __attribute__((always_inline)) {
    if constexpr ((EPI & WS_KMASK) != 0)  // row clamped: the last tile's rows past M read row M - 1's word
      m = a.kmask[min((int64_t)t * WS_ROWS + (lane & 31), M - 1) * 4 + wave];
  };
  auto e1 = [&](const floatx16& p1, int j, int part, int tp) __attribute__((always_inline)) {
    const int rl = (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
    if (part == 0) {
      float x = fmaf(p1[j], cs, bv);
      if constexpr ((EPI & WS_RELU) != 0) x = fmaxf(x, 0.f);
      xv[j] = x;
    } else if (part == 1) {
      if constexpr ((EPI & WS_DROP) != 0 && (EPI & WS_KMASK) != 0) {
        // the keep bits K1 computed for this tile's rows: lane r < 32 holds row r's word of this
        // wave's 32 columns (== keep_elem(seed, row·Nc + col), bit for bit)
        const uint32_t bits = (uint32_t)__shfl((int)mku, rl);
        xv[j] = ((bits >> (lane & 31)) & 1u) ? xv[j] * a.drop_scale : 0.f;
      } else if constexpr ((EPI & WS_DROP) != 0) {
        const uint32_t h0 = ((uint32_t)(tp * WS_ROWS + 4 * (lane >> 5)) * (uint32_t)Nc + (uint32_t)col) * kDropGolden +
                            (uint32_t)seed;
        xv[j] = keep_premixed(h0 + (uint32_t)(rl - 4 * (lane >> 5)) * hstep, seed, a.keep_thresh) ? xv[j] * a.drop_scale
                                                                                                  : 0.f;
      }
    } else {
      CT[rl * BN + col] = colok ? xv[j] : 0.f;
    }
  };
  float4 cv[4];
  float4 ph[2][4];
  float pacc0 = 0.f, pacc1 = 0.f;
  constexpr int NP = 2;
  const int ppart = tid % NP, pq = (tid / NP) % MAXPROJ, prl = tid / (NP * MAXPROJ);
  auto c_read = [&](int i) __attribute__((always_inline)) {
    const int u = tid + 256 * i;
    cv[i] = *reinterpret_cast<const float4*>(CT + (u / (BN / 4)) * BN + (u % (BN / 4)) * 4);
  };
  auto c_store = [&](int i, int tp) __attribute__((always_inline)) {
    const int u = tid + 256 * i;
    const int rl = u / (BN / 4), c4 = (u % (BN / 4)) * 4;
    const u32x4 xv4 = {__float_as_uint(cv[i].x), __float_as_uint(cv[i].y), __float_as_uint(cv[i].z),
                       __float_as_uint(cv[i].w)};
    const uint32_t off = (c4 < Nc && tp >= 0) ? (uint32_t)((((int64_t)tp * WS_ROWS + rl) * ldc + c4) * 4) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b128(xv4, crsrc, (int)off, 0, 0);
  };
  auto p_read = [&](int tt) __attribute__((always_inline)) {
    const float4* hrow = reinterpret_cast<const float4*>(CT + prl * BN);
    const float4* prw = reinterpret_cast<const float4*>(PL + pq * PLP);
    const int j = ppart + 2 * NP * tt;
    ph[tt & 1][0] = hrow[j];
    ph[tt & 1][1] = prw[j];
    ph[tt & 1][2] = hrow[j + NP];
    ph[tt & 1][3] = prw[j + NP];
  };
  auto p_fma = [&](int tt) __attribute__((always_inline)) {
    const float4 h0_ = ph[tt & 1][0], p0 = ph[tt & 1][1], h1_ = ph[tt & 1][2], p1 = ph[tt & 1][3];
    pacc0 = fmaf(h0_.x, p0.x, pacc0); pacc0 = fmaf(h0_.y, p0.y, pacc0);
    pacc0 = fmaf(h0_.z, p0.z, pacc0); pacc0 = fmaf(h0_.w, p0.w, pacc0);
    pacc1 = fmaf(h1_.x, p1.x, pacc1); pacc1 = fmaf(h1_.y, p1.y, pacc1);
    pacc1 = fmaf(h1_.z, p1.z, pacc1); pacc1 = fmaf(h1_.w, p1.w, pacc1);
  };
  auto p_done = [&](int tp) __attribute__((always_inline)) {
    float zsum = pacc0 + pacc1;
    zsum += __shfl_xor(zsum, 1);
    pacc0 = pacc1 = 0.f;
    const int64_t row = (int64_t)tp * WS_ROWS + prl;
    const uint32_t zoff = (ppart == 0 && pq < a.nproj && tp >= 0) ? (uint32_t)((row * a.ldz + pq) * 4) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(zsum), zrsrc, (int)zoff, 0, 0);
  };
  constexpr int PTRIPS = BN / 4 / (2 * NP);
  constexpr int NE2 = 8 + 2 * PTRIPS + 1;
  auto e2 = [&](int q, int tp) __attribute__((always_inline)) {
    if (q < 4) c_read(q);
    else if (q < 8) c_store(q - 4, tp);
    else if constexpr ((EPI & WS_PROJ) != 0) {
      const int k = q - 8;
      if (k == 0) p_read(0);
      else if (k < 2 * PTRIPS - 1) {
        if (k & 1) p_read((k + 1) / 2);
        else p_fma(k / 2 - 1);
      } else if (k == 2 * PTRIPS - 1) {
        p_fma(PTRIPS - 1);
      } else if (k == 2 * PTRIPS) {
        p_done(tp);
      }
    }
  };

  constexpr h2s::Sched SC = h2s::make(QP, NE2, NSL);
  auto slot = [&](auto kc, char* nxt, const floatx16& p1, int tp, int t) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    static_for<SC.first[k + 1] - SC.first[k]>([&](auto ac) __attribute__((always_inline)) {
      constexpr int ai = SC.first[k] + decltype(ac)::value;
      constexpr int kind = SC.kind[ai], i = SC.idx[ai];
      if constexpr (kind == h2s::E1) {
        if constexpr (!(LAB & 2)) e1(p1, i / 3, i % 3, tp);
      } else if constexpr (kind == h2s::E2) {
        if constexpr (!(LAB & 2)) e2(i, tp);
      } else if constexpr (kind == h2s::SP) {
        if constexpr (!(LAB & 4)) put_piece(nxt, i);
      } else if constexpr (kind == h2s::SL) {
        if constexpr (!(LAB & 4)) load_piece(i, t + 2 * (int)gridDim.x);
      } else if constexpr (kind == h2s::BAR) {
        __syncthreads();  // every wave's E1 is in the C tile
      }
    });
  };
#define NTH_FENCE __builtin_amdgcn_sched_barrier(0)
  auto kloop = [&](const char* cur, char* nxt, floatx16& c1, const floatx16& p1, int t, int tp, uint32_t& mkl,
                   uint32_t mkp) __attribute__((always_inline)) {
    mku = mkp;  // E1 of tile tp reads its keep bits
    uint32_t mkraw = 0u;
    load_mk(mkraw, t);  // tile t's, for its E1 one tile later
    f16x8 x[2];
    auto frag = [&](int s, int p) __attribute__((always_inline)) { return *reinterpret_cast<const f16x8*>(cur + p * PLB + s * WS_KSB + foff); };
    x[0] = frag(0, 0);
    x[1] = frag(0, 1);
    static_for<NKS>([&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      // small terms first: A_hi·B_lo, A_lo·B_hi, then A_hi·B_hi'
      NTH_FENCE;
      if constexpr (!(LAB & 1)) h2_mfma<s == 0>(c1, x[0], bw[s][2]);
      NTH_FENCE;
      slot(std::integral_constant<int, 3 * s>{}, nxt, p1, tp, t);
      NTH_FENCE;
      if constexpr (!(LAB & 1)) h2_mfma<0>(c1, x[1], bw[s][1]);
      NTH_FENCE;
      if constexpr (s + 1 < NKS) x[1] = frag(s + 1, 1);
      slot(std::integral_constant<int, 3 * s + 1>{}, nxt, p1, tp, t);
      NTH_FENCE;
      if constexpr (!(LAB & 1)) h2_mfma<0>(c1, x[0], bw[s][0]);
      NTH_FENCE;
      if constexpr (s + 1 < NKS) x[0] = frag(s + 1, 0);
      slot(std::integral_constant<int, 3 * s + 2>{}, nxt, p1, tp, t);
    });
    NTH_FENCE;
    if constexpr ((EPI & WS_KMASK) != 0) {
      // consume the keep-bit load HERE, at the end of the chain that issued it: the wait hipcc
      // places before this copy counts only the loads issued after it (landed long since); a
      // first use in the next tile's E1 made it wait for the A prefetches issued in between
      asm volatile("v_mov_b32 %0, %1" : "=v"(mkl) : "v"(mkraw));
    }
    if constexpr ((LAB & 1) != 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) c1[r] = (float)x[0][r & 7];
    }
    h2_mfma_end(c1);
  };
#undef NTH_FENCE
  auto finish = [&](const floatx16& p1, int tp) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 48; ++k) e1(p1, k / 3, k % 3, tp);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NE2; ++q) e2(q, tp);
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;
#pragma unroll
  for (int i = 0; i < QP; ++i) load_piece(i, t);
#pragma unroll
  for (int i = 0; i < QP; ++i) put_piece(A0, i);
#pragma unroll
  for (int i = 0; i < QP; ++i) load_piece(i, t + G);
  floatx16 aA, aB;
#pragma unroll
  for (int r = 0; r < 16; ++r) aA[r] = aB[r] = 0.f;
  __syncthreads();
  int tp = -1;
  while (true) {
    kloop(A0, A1, aA, aB, t, tp, mk[0], mk[1]);
    __syncthreads();
    tp = t;
    t += G;
    if (t >= ntiles) {
      mku = mk[0];
      finish(aA, tp);
      break;
    }
    kloop(A1, A0, aB, aA, t, tp, mk[1], mk[0]);
    __syncthreads();
    tp = t;
    t += G;
    if (t >= ntiles) {
      mku = mk[1];
      finish(aB, tp);
      break;
    }
  }
}

// B image of the half-pair NT (gemm_common.hpp ws_prep_h2_cols): the standalone launch, one wave
// per output column (BN / 16 blocks of 1024).  (K1 can also carry it: gnn_sage_mean_fwd_h2's prep_b.)
constexpr int WS_PREP_GRID = BN / (WS_PREP_THREADS / 64);
__global__ __launch_bounds__(WS_PREP_THREADS) void ws_prep_h2_kernel(H2Prep p) {
  ws_prep_h2_cols<WS_PREP_THREADS>(p, (int)blockIdx.x);
}

// ---------------------------------------------------------------- bf16 image form (K7a-b)
// bf16 storage (BASELINE configs[4]): A is a bf16 image [M][ld] (one plane; ld = 16·NKS; A1 in
// columns [0, k1), A2 in [col2, col2 + k2), zeros elsewhere), B the Linear weights rounded to bf16
// (plane 0 of the ws B image: RNE(W)), C bf16.  One product per MFMA, so the kernel is HBM-bound
// (A once, C once) and its staging is an LDS-DMA ring: every 1 KB k-step block of a 32-row tile is
// ONE global_load_lds_dwordx4 (lane l: row l/2, k-half (l & 1) ^ bit 3 of the row — the fragment
// layout above, lane-linear), NBUF tile buffers with NBUF - 1 tiles in flight across each raw
// s_barrier (counted vmcnt: the DMA and the E2 stores are the loop's only vector-memory ops).
// One 256-thread block per CU sweeps tiles t = blockIdx.x, += gridDim.x; wave w owns columns
// 32w .. +32 with its B fragments stationary in VGPRs.  Per tile:
//   wait for its DMA, barrier | E2 of the previous tile from its C tile: coalesced 16-byte bf16 C
//   row stores and the projection z = h·Pᵀ of the ROUNDED h | DMA of tile + NBUF - 1 | NKS MFMAs
//   | E1: bias, ReLU, counter-hash dropout, bf16 rounding -> this tile's C tile (two, alternating).
// All LDS in one array (a second __shared__ object can make hipcc wait vmcnt(0) at ds_reads).
template <int NKS, int EPI, int NBUF>
__global__ __launch_bounds__(256) void gemm_nt_img16_kernel(NTArgs a, const uint4* __restrict__ bimg, int ntiles) {
  constexpr int QW = (NKS + 3) / 4;             // DMA instructions per wave per tile (uniform count)
  constexpr int ABUF = NKS * WS_KSB;
  constexpr int SCR = NBUF * ABUF;              // 1 KB target of the count-padding DMAs
  constexpr int CT0 = SCR + 1024;               // two C tiles [32][BN] f32
  constexpr int CTB = WS_ROWS * BN * 4;
  constexpr int LDSB = CT0 + 2 * CTB;
  constexpr bool PROJ = (EPI & WS_PROJ) != 0;
  constexpr int S = 2 + (PROJ ? 1 : 0);         // E2's stores per thread
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: the DMA targets are wave-uniform
  const int64_t M = a.M;
  const int Nc = a.Nc;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;

  // ---- stationary B: columns 32·wave .. +32, all k-steps, plane 0
  bf16x8 bw[NKS];
  {
    const int slot = 2 * (32 * wave + (lane & 31)) + (lane >> 5);
#pragma unroll
    for (int s = 0; s < NKS; ++s) bw[s] = __builtin_bit_cast(bf16x8, bimg[(s * 3) * 256 + slot]);
  }
  // ---- the LDS-DMA of one tile (rows clamped into the image: tail rows repeat row M - 1 and
  //      their C rows are dropped by the store range)
  const int ld = a.ap_ld;
  const int prow = lane >> 1;
  const int khalf = (lane & 1) ^ ((prow >> 3) & 1);
  // The DMA is an asm statement (M0 written in the same statement): hipcc's waitcnt pass cannot
  // tell DMA targets from the C-tile and fragment reads in the one LDS array and would drain every
  // DMA (vmcnt(0)) at the first ds_read after each barrier; hidden from it, only the counted
  // waits below order the ring.
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto glds16 = [](const uint16_t* src, uint32_t dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  auto dma = [&](int tt, int buf) {
    const int tc = min(tt, ntiles - 1);
    const int64_t row = min((int64_t)tc * WS_ROWS + prow, M - 1);
    const uint16_t* src = a.ap + row * ld + 8 * khalf;
#pragma unroll
    for (int i = 0; i < QW; ++i) {
      const int b = wave + 4 * i;
      if (b < NKS) glds16(src + 16 * b, lds0 + (uint32_t)(buf * ABUF + b * WS_KSB));
      else glds16(src, lds0 + (uint32_t)SCR);
    }
  };
  // vmcnt(N) alone (expcnt / lgkmcnt at their maxima), gfx9 encoding
  auto wait_vm = [](auto nc) {
    constexpr int N = decltype(nc)::value;
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  };

  const int frow = lane & 31;
  const uint32_t foff = (uint32_t)(frow * 32 + (((lane >> 5) ^ ((frow >> 3) & 1)) << 4));
  const int col = 32 * wave + (lane & 31);
  const bool colok = col < Nc;
  const uint32_t hstep = (uint32_t)Nc * kDropGolden;
  // projection: this thread's row of the C tile and column slice, its P[q][slice] in registers
  const int prow8 = tid >> 3, pcb = tid & 7;
  float preg[MAXPROJ][16];
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = 16 * pcb + j;
      preg[q][j] = (PROJ && q < a.nproj && c < Nc) ? a.proj[(int64_t)q * Nc + c] : 0.f;
    }
  float bv = 0.f;
  if constexpr ((EPI & WS_BIAS) != 0) bv = colok ? a.bias[col] : 0.f;
  const int64_t ldc = a.ldc;
  const __amdgpu_buffer_rsrc_t crsrc = __builtin_amdgcn_make_buffer_rsrc(a.c, 0, (int)(M * ldc * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t zrsrc =
      __builtin_amdgcn_make_buffer_rsrc(a.z, 0, PROJ ? (int)(M * a.ldz * 4) : 0, 0x00020000);

  // E1: the tile's accumulators -> C tile (bias, ReLU, dropout, bf16 rounding)
  auto e1 = [&](const floatx16& acc, int tt, float* ct) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int rl = (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
      float x = acc[j] + bv;
      if constexpr ((EPI & WS_RELU) != 0) x = fmaxf(x, 0.f);
      if constexpr ((EPI & WS_DROP) != 0) {  // == keep_elem(seed, row·Nc + col), bit for bit
        const uint32_t h0 = ((uint32_t)(tt * WS_ROWS) * (uint32_t)Nc + (uint32_t)col) * kDropGolden + (uint32_t)seed;
        x = keep_premixed(h0 + (uint32_t)rl * hstep, seed, a.keep_thresh) ? x * a.drop_scale : 0.f;
      }
      const uint32_t hb = ws_pk(x, 0.f) & 0xffffu;  // RNE to bf16: what C stores
      ct[rl * BN + col] = colok ? __uint_as_float(hb << 16) : 0.f;
    }
  };
  // E2: coalesced bf16 C rows (16 columns of 8 per row, 2 per thread) and the projection
  auto e2 = [&](int tp, const float* ct) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int u = tid + 256 * q;
      const int rl = u >> 4, c8 = (u & 15) * 8;
      const float4 v0 = *reinterpret_cast<const float4*>(ct + rl * BN + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(ct + rl * BN + c8 + 4);
      const u32x4 w = {ws_pk(v0.x, v0.y), ws_pk(v0.z, v0.w), ws_pk(v1.x, v1.y), ws_pk(v1.z, v1.w)};
      const uint32_t off = (c8 < Nc && tp >= 0) ? (uint32_t)((((int64_t)tp * WS_ROWS + rl) * ldc + c8) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(w, crsrc, (int)off, 0, 0);
    }
    if constexpr (PROJ) {  // thread: row tid / 8, columns 16·(tid % 8) .. +16 (its P slice in registers)
      const float* hr = ct + prow8 * BN + 16 * pcb;
      float zq[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const float4 h = *reinterpret_cast<const float4*>(hr + 4 * c4);
#pragma unroll
        for (int q = 0; q < MAXPROJ; ++q) {
          zq[q] = fmaf(h.x, preg[q][4 * c4 + 0], zq[q]);
          zq[q] = fmaf(h.y, preg[q][4 * c4 + 1], zq[q]);
          zq[q] = fmaf(h.z, preg[q][4 * c4 + 2], zq[q]);
          zq[q] = fmaf(h.w, preg[q][4 * c4 + 3], zq[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) {  // the 8 column slices of the row: fixed xor tree
        zq[q] += __shfl_xor(zq[q], 1);
        zq[q] += __shfl_xor(zq[q], 2);
        zq[q] += __shfl_xor(zq[q], 4);
      }
      const u32x4 zw = {__float_as_uint(zq[0]), __float_as_uint(zq[1]), __float_as_uint(zq[2]), __float_as_uint(zq[3])};
      const uint32_t zoff = (pcb == 0 && tp >= 0) ? (uint32_t)((((int64_t)tp * WS_ROWS + prow8) * a.ldz) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(zw, zrsrc, (int)zoff, 0, 0);
    }
  };

  // B, bias, projection and seed loads landed before the ring starts (hipcc would otherwise wait
  // for them inside the loop with counts that also drain the DMAs)
  wait_vm(std::integral_constant<int, 0>{});
  // prologue: tiles t, t + G, .. in flight
#pragma unroll
  for (int b = 0; b < NBUF - 1; ++b) dma(t + b * G, b);
  int tp = -1;
  for (int i = 0;; ++i) {
    // DMA(i) done: after it were issued the prologue's later DMAs and, per iteration since, S
    // stores + one tile's DMA
    if (i == 0) wait_vm(std::integral_constant<int, (NBUF - 2) * QW>{});
    else if (NBUF == 3 || i == 1) wait_vm(std::integral_constant<int, (NBUF - 2) * QW + S>{});
    else wait_vm(std::integral_constant<int, (NBUF - 2) * QW + (NBUF - 2) * S>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous E1's C-tile writes
    __builtin_amdgcn_s_barrier();
    e2(tp, reinterpret_cast<const float*>(smem + CT0 + ((i + 1) & 1) * CTB));
    dma(t + (NBUF - 1) * G, (i + NBUF - 1) % NBUF);
    const char* cur = smem + (i % NBUF) * ABUF;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(cur + s * WS_KSB + foff);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, bw[s], acc, 0, 0, 0);
    }
    e1(acc, t, reinterpret_cast<float*>(smem + CT0 + (i & 1) * CTB));
    tp = t;
    t += G;
    if (t >= ntiles) {
      wait_vm(std::integral_constant<int, 0>{});  // no DMA may outlive the block's LDS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      e2(tp, reinterpret_cast<const float*>(smem + CT0 + (i & 1) * CTB));
      break;
    }
  }
}

int ws_num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// The last (partial) row tile, zero-padded to 32 rows: [32][k1] then [32][k2] f32.
__device__ __forceinline__ void ws_tail_block(const NTArgs& a, float* __restrict__ tail, int64_t r0, int blk) {
  const int n1 = WS_ROWS * a.k1, n = n1 + WS_ROWS * a.k2;
  {
    const int i = blk * 256 + threadIdx.x;  // one element per thread
    if (i >= n) return;
    const bool s2 = i >= n1;
    const int kg = s2 ? a.k2 : a.k1;
    const int j = s2 ? i - n1 : i;
    const int r = j / kg, c = j - r * kg;
    const int64_t row = r0 + r;
    tail[i] = row < a.M ? (s2 ? a.a2[row * a.lda2 + c] : a.a1[row * a.lda1 + c]) : 0.f;
  }
}

// B image over the CONCATENATED K (k < k1: W1, else W2 at k - k1): per 16-deep chunk c,
// [plane hi/mid/lo][2n + khalf] uint4 (8 bf16), zero for n >= Nc and k >= k1 + k2.
// col2: first K index of W2 (k1, or the split image's ap_col2 with zeros in between)
__device__ __forceinline__ void ws_presplit_block(const NTArgs& a, uint4* __restrict__ img, int nchunks, int blk,
                                                  int col2) {
  const int idx = blk * 256 + threadIdx.x;  // (chunk, n, khalf)
  if (idx >= nchunks * 256) return;
  const int c = idx >> 8, n = (idx & 255) >> 1, kh = idx & 1;
  float e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * c + 8 * kh + j;
    float v = 0.f;
    if (n < a.Nc && k < a.k1) v = a.w1[(int64_t)n * a.ldw1 + k];
    else if (n < a.Nc && k >= col2 && k < col2 + a.k2) v = a.w2[(int64_t)n * a.ldw2 + (k - col2)];
    e[j] = v;
  }
  uint32_t w[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j) ws_split(e[2 * j], e[2 * j + 1], w[j][0], w[j][1], w[j][2]);
#pragma unroll
  for (int p = 0; p < 3; ++p) img[((int64_t)c * 3 + p) * 256 + (idx & 255)] = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
}

// One launch for both per-call preparations (blocks [0, nchunks): B image; the rest: tail tile).
__global__ __launch_bounds__(256) void ws_prep_kernel(NTArgs a, uint4* __restrict__ img, int nchunks,
                                                      float* __restrict__ tail, int64_t r0, int col2) {
  if ((int)blockIdx.x < nchunks) ws_presplit_block(a, img, nchunks, blockIdx.x, col2);
  else ws_tail_block(a, tail, r0, blockIdx.x - nchunks);
}

template <int NKS, int KS>
void launch_ws_k(const NTArgs& a, const uint4* bimg, const float* tail, hipStream_t st) {
  const int ntiles = (int)ceil_div(a.M, WS_ROWS);
  const int grid = std::min(ntiles, ws_num_cus());
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
#define GNN_WS(E) gemm_nt_ws_kernel<NKS, E, KS><<<grid, 256 * KS, 0, st>>>(a, bimg, ntiles, tail)
  if (proj && drop) GNN_WS(WS_BIAS | WS_RELU | WS_DROP | WS_PROJ);
  else if (proj) GNN_WS(WS_BIAS | WS_RELU | WS_PROJ);
  else if (drop) GNN_WS(WS_BIAS | WS_RELU | WS_DROP);
  else if (relu) GNN_WS(WS_BIAS | WS_RELU);
  else if (bias) GNN_WS(WS_BIAS);
  else GNN_WS(0);
#undef GNN_WS
}

}  // namespace

// Shapes the weight-stationary form takes: f32 A and C, contiguous A segments (lda == k, even k,
// 16-byte aligned), 64 < N <= 128, M >= 32, ceil((k1 + k2) / 16) k-steps in {8, 11, 16, 21}, and
// an epilogue among plain | bias | bias+ReLU | bias+ReLU+dropout, each + projection when ReLU.
bool nt_ws_ok(const NTArgs& a) {
  if (a.a_bf16 || a.c_bf16 || !a.w1 || a.Nc > BN || a.Nc < 1) return false;
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (a.lda1 != a.k1 || (a.k1 & 1) || !al(a.a1)) return false;
  // buffer-store epilogue: 16-byte C rows, whole float4 column chunks, 31-bit byte offsets
  if (a.c && (!al(a.c) || a.ldc % 4 != 0 || a.M * a.ldc * 4 >= ((int64_t)1 << 31))) return false;
  if (a.Nc % 4 != 0 || (a.nproj > 0 && a.M * a.ldz * 4 >= ((int64_t)1 << 31))) return false;
  if (a.k2 > 0 && (a.lda2 != a.k2 || (a.k2 & 1) || !al(a.a2))) return false;
  const int nks = (a.k1 + a.k2 + 15) / 16;
  if (nks != 8 && nks != 11 && nks != 16 && nks != 21) return false;
  if (a.M < WS_ROWS || a.M * (int64_t)std::max(a.k1, a.k2) >= ((int64_t)1 << 40)) return false;
  // the block always computes 128 columns: at N <= 64 half its MFMAs are wasted and the tiled
  // x3 kernel wins (r07: GAT/GCN layer 1, K = 166, N = 64: 104 vs 80 us)
  if (a.Nc <= 64) return false;  // (r22: also slower on SAGE-ResBN's K = 128, N = 64 GEMMs: 1.070 vs 1.053 ms/step)
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
  if ((drop || proj || relu) && !(relu && bias)) return false;
  return true;
}

size_t nt_ws_tail_offset(int64_t k1, int64_t k2) {  // the B image (<= 24 chunks x 12 KB), then the tail tile
  return (size_t)((k1 + k2 + 15) / 16) * 3 * 256 * sizeof(uint4);
}

void launch_nt_ws(const NTArgs& a, uint4* img, hipStream_t st) {
  const int nks = (a.k1 + a.k2 + 15) / 16;
  float* tail = reinterpret_cast<float*>(reinterpret_cast<char*>(img) + nt_ws_tail_offset(a.k1, a.k2));
  ws_prep_kernel<<<(unsigned)(nks + ceil_div(WS_ROWS * (a.k1 + a.k2), 256)), 256, 0, st>>>(
      a, img, nks, tail, (ceil_div(a.M, WS_ROWS) - 1) * WS_ROWS, a.k1);
  // K parts per column group: 2 when the half-K B fragments and the rest fit a 256-register wave
  // without spills (NKS <= 16), 1 for NKS = 21 (252 AGPRs of B)
  switch (nks) {
    case 8: launch_ws_k<8, 2>(a, img, tail, st); break;
    case 11: launch_ws_k<11, 2>(a, img, tail, st); break;
    case 16: launch_ws_k<16, 2>(a, img, tail, st); break;
    default: launch_ws_k<21, 1>(a, img, tail, st); break;
  }
}

}  // namespace gnnmp

namespace gnnmp {

// The split-image form: f32 C, the w1/w2 B form, A from NTArgs::ap with a 336-wide image row
// (21 k-steps: the SAGE layer-1 [agg | x] of 166 + 166 features, each padded to 168),
// 64 < N <= 128, M >= 32, the nt_ws_ok epilogues.
bool nt_planes_ok(const NTArgs& a) {
  // 336-wide rows (the SAGE [agg | x]) for 64 < N <= 128; 176-wide rows (one 166-wide input, the
  // GCN / GAT layer-1 x) for any N <= 128 (N <= 64 leaves half the MFMA columns zero: the kernel
  // is bound by its A stream there, not by the MFMA chain)
  if (!a.ap || a.ap_h2 || a.a_bf16 || a.c_bf16 || !a.w1 || (a.k2 > 0 && !a.w2) || a.Nc > BN || a.Nc < 1) return false;
  if (!(a.ap_ld == 336 && a.Nc > 64) && a.ap_ld != 176) return false;
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al(a.ap) || a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 || a.ap_col2 + a.k2 > a.ap_ld)
    return false;
  if (a.ap_ps < a.M * (int64_t)a.ap_ld || 3 * a.ap_ps * 2 >= ((int64_t)1 << 31)) return false;
  if (a.c && (!al(a.c) || a.ldc % 4 != 0 || a.M * a.ldc * 4 >= ((int64_t)1 << 31))) return false;
  if (a.Nc % 4 != 0 || (a.nproj > 0 && a.M * a.ldz * 4 >= ((int64_t)1 << 31))) return false;
  if (a.M < WS_ROWS) return false;
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
  if ((drop || proj || relu) && !(relu && bias)) return false;
  return true;
}

// The half-pair form: f32 C, the w1/w2 B form, a half-pair image row of 336 (21 k-steps: the
// SAGE layer-1 [agg | x]) or 176 (11: one input, the GCN / GAT layer-1 x), 1 <= N <= 128 with
// N % 4 == 0, M >= 32, the nt_ws_ok epilogues.
bool nt_h2_ok(const NTArgs& a) {
  if (!a.ap || !a.ap_h2 || a.a_bf16 || a.c_bf16 || !a.w1 || (a.k2 > 0 && !a.w2) || a.Nc > BN || a.Nc < 1) return false;
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if ((a.ap_ld != 336 && a.ap_ld != 176) || !al(a.ap) || a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 || a.ap_col2 + a.k2 > a.ap_ld)
    return false;
  if (a.ap_ps < a.M * (int64_t)a.ap_ld || 2 * a.ap_ps * 2 >= ((int64_t)1 << 31)) return false;
  if (a.c && (!al(a.c) || a.ldc % 4 != 0 || a.M * a.ldc * 4 >= ((int64_t)1 << 31))) return false;
  if (a.Nc % 4 != 0 || (a.nproj > 0 && a.M * a.ldz * 4 >= ((int64_t)1 << 31))) return false;
  if (a.M < WS_ROWS) return false;
  // the prep kernel's linear sweep indexes the weights with 32-bit element offsets
  if (a.ldw1 < a.k1 || a.Nc * a.ldw1 >= ((int64_t)1 << 30) || (a.w2 && a.k2 > 0 && (a.ldw2 < a.k2 || a.Nc * a.ldw2 >= ((int64_t)1 << 30))))
    return false;
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
  if ((drop || proj || relu) && !(relu && bias)) return false;
  return true;
}

H2Prep h2_prep_of(const NTArgs& a, uint4* img) {
  H2Prep p{};
  p.w1 = a.w1; p.w2 = a.w2; p.ldw1 = a.ldw1; p.ldw2 = a.ldw2;
  p.k1 = a.k1; p.k2 = a.k2; p.Nc = a.Nc; p.col2 = a.ap_col2;
  p.blocks = a.ap_ld / 16;
  p.img = img;
  p.colscale = reinterpret_cast<float*>(img + p.blocks * 3 * 256);
  p.a_unscale = ldexpf(1.0f, -a.ap_exp);  // |ap_exp| <= 100 (gemm_nt_dispatch): a normal float
  return p;
}

void launch_prep_h2(const H2Prep& p, hipStream_t st) {
  ws_prep_h2_kernel<<<WS_PREP_GRID, WS_PREP_THREADS, 0, st>>>(p);
}

// workspace: the B image (NKS k-steps x 3 planes x 256 slots x 16 B), then the 128 column scales
template <int NKS>
void launch_nt_h2_k(const NTArgs& a, uint4* img, hipStream_t st, int phase) {
  float* colscale = reinterpret_cast<float*>(img + NKS * 3 * 256);
  if (phase & NT_PHASE_PREP) ws_prep_h2_kernel<<<WS_PREP_GRID, WS_PREP_THREADS, 0, st>>>(h2_prep_of(a, img));
  if (!(phase & NT_PHASE_RUN)) return;
  const int ntiles = (int)ceil_div(a.M, WS_ROWS);
  // as many blocks as the tiles per block that one block per CU gives need: a shard's 850 tiles run
  // on 213 blocks of 4 (not 256 blocks of 3 or 4: the same longest block, 17 % fewer B loads)
  const int per = (int)ceil_div(ntiles, ws_num_cus());
  const int grid = (int)ceil_div(ntiles, per);
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
#define GNN_NH(E) gemm_nt_h2_kernel<NKS, E><<<grid, 256, 0, st>>>(a, img, colscale, ntiles)
  if (proj && drop && a.kmask) GNN_NH(WS_BIAS | WS_RELU | WS_DROP | WS_PROJ | WS_KMASK);
  else if (drop && a.kmask) GNN_NH(WS_BIAS | WS_RELU | WS_DROP | WS_KMASK);
  else if (proj && drop) GNN_NH(WS_BIAS | WS_RELU | WS_DROP | WS_PROJ);
  else if (proj) GNN_NH(WS_BIAS | WS_RELU | WS_PROJ);
  else if (drop) GNN_NH(WS_BIAS | WS_RELU | WS_DROP);
  else if (relu) GNN_NH(WS_BIAS | WS_RELU);
  else if (bias) GNN_NH(WS_BIAS);
  else GNN_NH(0);
#undef GNN_NH
}

void launch_nt_h2(const NTArgs& a, uint4* img, hipStream_t st, int phase) {
  if (a.ap_ld == 176) launch_nt_h2_k<11>(a, img, st, phase);
  else launch_nt_h2_k<21>(a, img, st, phase);
}

// The bf16 image form: bf16 A image (one plane, ld 256 or 336), bf16 C, the w1/w2 B form,
// 8 <= N <= 128 (N % 8 == 0), M >= 32, the nt_ws_ok epilogues.
bool nt_img16_ok(const NTArgs& a) {
  if (!a.ap || a.ap_h2 || !a.a_bf16 || !a.c_bf16 || !a.c || !a.w1 || (a.k2 > 0 && !a.w2) || a.Nc > BN || a.Nc < 8 || a.Nc % 8)
    return false;
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al(a.ap) || (a.ap_ld != 256 && a.ap_ld != 336) || a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 ||
      a.ap_col2 + a.k2 > a.ap_ld)
    return false;
  if (!al(a.c) || a.ldc % 8 != 0 || a.ldc < a.Nc || a.M * a.ldc * 2 >= ((int64_t)1 << 31)) return false;
  // the projection is stored as one 16-byte z row: all four products, 16-byte aligned rows
  if (a.nproj > 0 && (a.nproj != MAXPROJ || a.ldz % 4 != 0 || !al(a.z) || a.M * a.ldz * 4 >= ((int64_t)1 << 31)))
    return false;
  if (a.M < WS_ROWS || ceil_div(a.M, WS_ROWS) >= INT32_MAX) return false;
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
  if ((drop || proj || relu) && !(relu && bias)) return false;
  return true;
}

template <int NKS>
void launch_nt_img16_k(const NTArgs& a, const uint4* img, hipStream_t st) {
  const int ntiles = (int)ceil_div(a.M, WS_ROWS);
  const int grid = std::min(ntiles, ws_num_cus());
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
#define GNN_I16(E) gemm_nt_img16_kernel<NKS, E, 4><<<grid, 256, 0, st>>>(a, img, ntiles)
  if (proj && drop) GNN_I16(WS_BIAS | WS_RELU | WS_DROP | WS_PROJ);
  else if (proj) GNN_I16(WS_BIAS | WS_RELU | WS_PROJ);
  else if (drop) GNN_I16(WS_BIAS | WS_RELU | WS_DROP);
  else if (relu) GNN_I16(WS_BIAS | WS_RELU);
  else if (bias) GNN_I16(WS_BIAS);
  else GNN_I16(0);
#undef GNN_I16
}

void launch_nt_img16(const NTArgs& a, uint4* img, hipStream_t st, int phase) {
  const int nks = a.ap_ld / 16;
  if (phase & NT_PHASE_PREP) ws_prep_kernel<<<(unsigned)nks, 256, 0, st>>>(a, img, nks, nullptr, 0, a.ap_col2);  // B image (plane 0 used)
  if (!(phase & NT_PHASE_RUN)) return;
  if (nks == 16) launch_nt_img16_k<16>(a, img, st);
  else launch_nt_img16_k<21>(a, img, st);
}

template <int NKS>
void launch_nt_ws_planes_k(const NTArgs& a, uint4* img, hipStream_t st) {
  const int ntiles = (int)ceil_div(a.M, WS_ROWS);
  const int grid = std::min(ntiles, ws_num_cus());
  const bool drop = a.dropout != 0, relu = a.relu != 0, bias = a.bias != nullptr, proj = a.nproj > 0;
#define GNN_WSP(E) gemm_nt_planes_kernel<NKS, E><<<grid, 256, 0, st>>>(a, img, ntiles)
  if (proj && drop) GNN_WSP(WS_BIAS | WS_RELU | WS_DROP | WS_PROJ);
  else if (proj) GNN_WSP(WS_BIAS | WS_RELU | WS_PROJ);
  else if (drop) GNN_WSP(WS_BIAS | WS_RELU | WS_DROP);
  else if (relu) GNN_WSP(WS_BIAS | WS_RELU);
  else if (bias) GNN_WSP(WS_BIAS);
  else GNN_WSP(0);
#undef GNN_WSP
}

void launch_nt_ws_planes(const NTArgs& a, uint4* img, hipStream_t st, int phase) {
  const int nks = a.ap_ld / 16;
  if (phase & NT_PHASE_PREP) ws_prep_kernel<<<(unsigned)nks, 256, 0, st>>>(a, img, nks, nullptr, 0, a.ap_col2);  // the B image only
  if (!(phase & NT_PHASE_RUN)) return;
  if (nks == 11) launch_nt_ws_planes_k<11>(a, img, st);
  else launch_nt_ws_planes_k<21>(a, img, st);
}

}  // namespace gnnmp
