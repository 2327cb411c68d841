// The small per-step work around the hot path, fused: the masked class-weighted cross entropy
// of src/train_gnn.py:136-183 (loss + dlogits in one pass over the N rows) and
// clip_grad_norm_ + Adam (src/train_gnn.py:203-206) over every parameter in two launches.
// Both replace chains of 6-12 small ATen kernels (index_select, log_softmax, nll_loss, their
// backward passes and zero fills; per-tensor norms, stack, clamp, mul, multi-tensor Adam).
// Reductions are fixed-order (block partials summed in index order): bitwise reproducible.
#include <algorithm>
#include <cmath>

#include "common.hpp"

namespace gnnmp {
namespace {

constexpr int kCeThreads = 256;
constexpr int kMaxClasses = 16;

__device__ __forceinline__ float block_sum(float v, float* sh) {
  // wave64 butterfly, then the 4 wave sums in order
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  return t;  // valid in thread 0
}

// loss_i = -w[y_i] · log_softmax(x_i)[y_i] on rows with mask_i (F.cross_entropy(weight=w,
// reduction='none')); dx_i = w[y_i] · (softmax(x_i) - onehot(y_i)) · inv_denom there, 0 elsewhere.
// partial[b] = Σ loss over block b's rows.  colsum (optional, ABI 21): colsum[b·C + c] = Σ dx[:, c]
// over block b's rows (the same fixed-order block sum): the output layer's bias gradient without
// a pass over dlogits (gnn_colsum_finish_f32 adds the blocks).
template <int CT>  // CT > 0: compile-time class count (registers); CT == 0: runtime C <= kMaxClasses
__global__ __launch_bounds__(kCeThreads) void masked_ce_kernel(int64_t N, int Crt, const float* __restrict__ x,
                                                               int64_t ldx, const int64_t* __restrict__ y,
                                                               const uint8_t* __restrict__ mask,
                                                               const float* __restrict__ w, float inv_denom,
                                                               float* __restrict__ dx, int64_t ldd,
                                                               float* __restrict__ partial,
                                                               float* __restrict__ colsum = nullptr) {
  constexpr int CM = CT > 0 ? CT : kMaxClasses;
  const int C = CT > 0 ? CT : Crt;
  __shared__ float sh[kCeThreads / 64];
  const int64_t row = (int64_t)blockIdx.x * kCeThreads + threadIdx.x;
  float l = 0.f;
  float dv[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) dv[c] = 0.f;
  if (row < N) {
    const int64_t t = y[row];
    const bool on = mask[row] != 0 && t >= 0 && t < C;
    float v[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) v[c] = c < C ? x[row * ldx + c] : 0.f;
    l = masked_ce_row<CM>(v, C, t, on, on ? w[t] : 0.f, inv_denom, dx + row * ldd, dv);
  }
  const float t = block_sum(l, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
  if (colsum) {  // kernel-uniform
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      if (c >= C) break;
      __syncthreads();  // sh reused
      const float s = block_sum(dv[c], sh);
      if (threadIdx.x == 0) colsum[(int64_t)blockIdx.x * C + c] = s;
    }
  }
}

// out[0] = scale · Σ_i partial[i], summed in a fixed order by one block.
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partial, int n, float scale,
                                                           float* __restrict__ out) {
  __shared__ float sh[4];
  float v = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) v += partial[i];
  const float t = block_sum(v, sh);
  if (threadIdx.x == 0) out[0] = t * scale;
}

// ---------------------------------------------------------------------------- clip + Adam
constexpr int kAdamThreads = 256;
constexpr int kAdamBlocks = 64;  // <= 64: clip_adam_kernel reduces the partials with one wave

struct AdamTable {
  int32_t n;
  float* p[GNN_ADAM_MAX_TENSORS];
  float* g[GNN_ADAM_MAX_TENSORS];
  float* m[GNN_ADAM_MAX_TENSORS];
  float* v[GNN_ADAM_MAX_TENSORS];
  int64_t off[GNN_ADAM_MAX_TENSORS + 1];  // element offsets of the flattened parameter list
};

// Σ g² over this block's slice of the flattened gradients, and the count of its non-finite
// elements (partial[kAdamBlocks + 1 + block]); block 0 also keeps the step count before this
// call in partial[kAdamBlocks] (clip_adam_kernel advances step[0] once it knows the step is
// taken: no block reads step[0] while another may write it).
// The block's tensor table staged in LDS once (the kernel-argument table indexed by a run-time
// tensor id compiled to a dependent load of the pointer per element), and a thread's elements of
// the block's slice (<= kAdamUnroll of them: all parameter lists of the path fit one pass at 64
// blocks) located by a walk in LDS, so every value load is issued before the first use.
constexpr int kAdamUnroll = 4;
struct AdamLds {
  int64_t off[GNN_ADAM_MAX_TENSORS + 1];
  float* p[GNN_ADAM_MAX_TENSORS];
  float* g[GNN_ADAM_MAX_TENSORS];
  float* m[GNN_ADAM_MAX_TENSORS];
  float* v[GNN_ADAM_MAX_TENSORS];
};
__device__ __forceinline__ void adam_stage(const AdamTable& tb, AdamLds& L) {
  const int t = threadIdx.x;
  if (t <= tb.n) L.off[t] = tb.off[t];
  if (t < tb.n) {
    L.p[t] = tb.p[t];
    L.g[t] = tb.g[t];
    L.m[t] = tb.m[t];
    L.v[t] = tb.v[t];
  }
  __syncthreads();
}
// tensor ids and in-tensor offsets of elements e, e + T, ... (valid[u] marks real ones; the others
// are clamped to the slice's LAST element, e1 - 1 >= every real one, so the walk only moves
// forward and every load stays inside a tensor)
template <int NTH = kAdamThreads>
__device__ __forceinline__ void adam_locate(const AdamLds& L, int n, int64_t e, int64_t e1, int (&j)[kAdamUnroll],
                                            int64_t (&i)[kAdamUnroll], bool (&valid)[kAdamUnroll]) {
  int jj = 0;
#pragma unroll
  for (int u = 0; u < kAdamUnroll; ++u) {
    const int64_t eu = e + (int64_t)u * NTH;
    valid[u] = eu < e1;
    const int64_t ec = valid[u] ? eu : e1 - 1;
    while (jj + 1 < n && ec >= L.off[jj + 1]) ++jj;
    j[u] = jj;
    i[u] = ec - L.off[jj];
  }
}

struct LossFinish {  // a deferred gnn_masked_ce_f32 loss (gnn_adam_group.loss_partial)
  const float* partial; int32_t n; float scale; float* out;
};
// *lf.out = lf.scale · Σ lf.partial: sum_partials_kernel's loop and reduction, exactly (one block)
__device__ __forceinline__ void finish_loss(const LossFinish& lf, float* sh) {
  float v = 0.f;
  for (int i = threadIdx.x; i < lf.n; i += kAdamThreads) v += threadIdx.x < kAdamThreads ? lf.partial[i] : 0.f;
  const float tl = block_sum(v, sh);
  if (threadIdx.x == 0) lf.out[0] = tl * lf.scale;
}

__global__ __launch_bounds__(kAdamThreads) void grad_sq_kernel(AdamTable tb, float* __restrict__ partial,
                                                                const float* __restrict__ step, LossFinish lf) {
  __shared__ float sh[kAdamThreads / 64];
  __shared__ AdamLds L;
  adam_stage(tb, L);
  const int64_t total = L.off[tb.n];
  const int64_t per = (total + gridDim.x - 1) / gridDim.x;
  const int64_t e0 = (int64_t)blockIdx.x * per, e1 = min(total, e0 + per);
  float s = 0.f, nf = 0.f;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kAdamUnroll * kAdamThreads) {
    int j[kAdamUnroll];
    int64_t i[kAdamUnroll];
    bool ok[kAdamUnroll];
    adam_locate(L, tb.n, e, e1, j, i, ok);
    float g[kAdamUnroll];
#pragma unroll
    for (int u = 0; u < kAdamUnroll; ++u) g[u] = L.g[j[u]][i[u]];
#pragma unroll
    for (int u = 0; u < kAdamUnroll; ++u) {  // in element order, as the one-at-a-time loop summed
      s = ok[u] ? fmaf(g[u], g[u], s) : s;
      nf += (ok[u] && !isfinite(g[u])) ? 1.f : 0.f;
    }
  }
  const float t = block_sum(s, sh);
  __syncthreads();  // sh reused
  const float tn = block_sum(nf, sh);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = t;
    partial[kAdamBlocks + 1 + blockIdx.x] = tn;
    if (blockIdx.x == 0) partial[kAdamBlocks] = step[0];
  }
  if (lf.partial && blockIdx.x == gridDim.x - 1) {
    __syncthreads();  // sh reused
    finish_loss(lf, sh);
  }
}

// Mirrors torch.optim.Adam's default (foreach, non-capturable) update: bias corrections and
// 1 - beta in double, as the Python scalars are; m.lerp_(g, 1 - b1); v = v·b2 + (1 - b2)·g·g;
// p += -lr/bc1 · m / (sqrt(v)/sqrt(bc2) + eps).
// skip_nonfinite (torch.amp.GradScaler.step's found_inf: some gradient ELEMENT is inf / NaN)
// leaves parameters, moments, gradients and the step count untouched.  A finite gradient whose
// Σg² overflows is not skipped: as in clip_grad_norm_, the norm is inf and the clip coefficient 0.
// partial: Σg² of block b at [b], its non-finite count at [nf_off + b], the step count before the
// update at [step_off]: grad_sq_kernel's layout (nblk = 64, nf_off = 65, step_off = 64) or the TN
// reduce's (ABI 20: nblk = nb, nf_off = nb, step_off = 2 nb).  Every block sums them in the same
// fixed order (lane-strided, then a butterfly per wave, then the 4 waves in order): for nblk <= 64
// that is grad_sq's one-wave butterfly exactly.
// SELF (NTH = 1024, gradients of at most kSelfMax = 2^15 elements): no partials — every block sums Σg² and
// the non-finite count over ALL the gradients itself, in one fixed order (thread t: elements
// t, t + NTH, ... in order, 16 loads in flight; then the wave butterflies and the waves in order),
// so every block holds the same norm and the grad_sq launch is saved.  The step count is read
// from *step at the start and written by the block that finishes last (a vector atomic on the
// workspace counter `done`, a running count mod kAdamBlocks): no block reads it after it changed.
constexpr int kSelfThreads = 1024;
// (GCN's 21.6k gradient elements: 10.0 us vs 7.1 + 7.2 in two launches; SAGE-ResBN's ~41k: 16.6
// vs 8.0 + 7.7 — the per-thread Σ passes grow with the count: profiles/r51_adam_one_launch.txt)
constexpr int64_t kSelfMax = 1 << 15;
static_assert(kSelfMax / 64 <= 4 * kSelfThreads, "a SELF block's Adam slice is one pass, loaded before the norm");
template <int NTH = kAdamThreads, bool SELF = false>
__global__ __launch_bounds__(NTH) void clip_adam_kernel(AdamTable tb, const float* __restrict__ partial,
                                                        int nblk, int nf_off, int step_off,
                                                        float* __restrict__ step,
                                                        double max_norm, double lr, double beta1,
                                                        double beta2, double eps, double wd,
                                                        float* __restrict__ norm_out, int skip_nonfinite,
                                                        int64_t* __restrict__ bump, LossFinish lf,
                                                        unsigned* __restrict__ done = nullptr) {
  __shared__ float coef_sh, snap_sh;
  __shared__ int skip_sh, last_sh;
  __shared__ float red_sh[2][NTH / 64];
  __shared__ AdamLds L;
  if (lf.partial && blockIdx.x == kAdamBlocks) {  // the extra block: a deferred CE loss, beside the update
    finish_loss(lf, &red_sh[0][0]);
    return;
  }
  if constexpr (SELF) {
    if (threadIdx.x == 0) snap_sh = step[0];  // (the LDS store waits for the load: complete before `done`)
  }
  adam_stage(tb, L);
  // this block's slice of the flattened parameters; its first pass's loads are issued here, before
  // the norm's reduction (they do not depend on it: one round trip less on the launch's path)
  const int64_t total = L.off[tb.n];
  const int64_t per = (total + kAdamBlocks - 1) / kAdamBlocks;  // (an extra loss block: no slice)
  const int64_t e0 = (int64_t)blockIdx.x * per, e1 = min(total, e0 + per);
  const bool has = e0 < e1;  // block-uniform
  int j[kAdamUnroll];
  int64_t i[kAdamUnroll];
  bool ok[kAdamUnroll];
  float g0[kAdamUnroll], p[kAdamUnroll], m0[kAdamUnroll], v0[kAdamUnroll];
  auto load_pass = [&](int64_t e) __attribute__((always_inline)) {
    adam_locate<NTH>(L, tb.n, e, e1, j, i, ok);
#pragma unroll
    for (int u = 0; u < kAdamUnroll; ++u) {  // every load of the pass issued first
      g0[u] = L.g[j[u]][i[u]];
      p[u] = L.p[j[u]][i[u]];
      m0[u] = L.m[j[u]][i[u]];
      v0[u] = L.v[j[u]][i[u]];
    }
  };
  if (has) load_pass(e0 + threadIdx.x);
  {
    float tot = 0.f, nf = 0.f;
    if constexpr (SELF) {  // Σg² over every gradient, this block's own fixed order
      constexpr int SU = 16;
      // the thread's elements increase, so the tensor walk only moves forward; the current tensor's
      // [lo, hi) and pointer stay in registers (LDS is read only when a boundary is crossed)
      int jj = 0;
      int64_t lo = 0, hi = L.off[1];
      const float* gp = L.g[0];
      for (int64_t q0 = threadIdx.x; q0 < total; q0 += (int64_t)SU * NTH) {
        float gv[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {  // every load of the pass issued first (clamped)
          const int64_t q = min(q0 + (int64_t)u * NTH, total - 1);
          while (q >= hi && jj + 1 < tb.n) {
            ++jj;
            lo = hi;
            hi = L.off[jj + 1];
            gp = L.g[jj];
          }
          gv[u] = gp[q - lo];
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const bool in = q0 + (int64_t)u * NTH < total;
          tot = in ? fmaf(gv[u], gv[u], tot) : tot;
          nf += (in && !isfinite(gv[u])) ? 1.f : 0.f;
        }
      }
    } else {
      constexpr int U = 4;  // every load of the first U·NTH partials issued before the sums (clamped, no branch)
      float pv[U], nv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = threadIdx.x + u * NTH, ic = min(i, nblk - 1);
        pv[u] = partial[ic];
        nv[u] = partial[nf_off + ic];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = threadIdx.x + u * NTH < nblk;
        tot += ok ? pv[u] : 0.f;
        nf += ok ? nv[u] : 0.f;
      }
      for (int i = threadIdx.x + U * NTH; i < nblk; i += NTH) {
        tot += partial[i];
        nf += partial[nf_off + i];
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      tot += __shfl_xor(tot, o);
      nf += __shfl_xor(nf, o);
    }
    // SELF: this thread's gradient loads (the Σ pass and its slice's first Adam pass) have landed
    // before the barrier behind which thread 0 counts the block as done (vmcnt(0))
    if constexpr (SELF) __builtin_amdgcn_s_waitcnt(0x0f70);
    if ((threadIdx.x & 63) == 0) {
      red_sh[0][threadIdx.x >> 6] = tot;
      red_sh[1][threadIdx.x >> 6] = nf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      tot = red_sh[0][0];
      nf = red_sh[1][0];
      for (int w = 1; w < NTH / 64; ++w) {
        tot += red_sh[0][w];
        nf += red_sh[1][w];
      }
      const float norm = sqrtf(tot);
      float coef = 1.0f;
      if (max_norm > 0.0) coef = fminf((float)max_norm / (norm + 1e-6f), 1.0f);  // torch clip_grad_norm_
      const bool skip = skip_nonfinite && nf > 0.f;
      coef_sh = coef;
      skip_sh = skip;
      if (blockIdx.x == 0) {
        if (norm_out) norm_out[0] = norm;
        if constexpr (!SELF) step[0] = partial[step_off] + (skip ? 0.0f : 1.0f);
        if (bump) bump[0] = bump[0] + 1;  // no kernel of this launch reads it
      }
      if constexpr (SELF) {  // every block has read *step (snap_sh) and every gradient: the last one
        // to get here advances the step.  The counter is never reset: each launch adds exactly
        // kAdamBlocks, so the block drawing old ≡ kAdamBlocks − 1 (mod kAdamBlocks) is the last one
        // whatever value a previous launch left (no reset store a torn-down launch could skip)
        last_sh = (atomicAdd(done, 1u) + 1u) % (unsigned)kAdamBlocks == 0u;
        if (last_sh) step[0] = snap_sh + (skip ? 0.0f : 1.0f);
      }
    }
  }
  __syncthreads();
  if (skip_sh) return;  // block-uniform
  if constexpr (SELF) {
    // clip_grad_norm_'s in-place scaling of .grad: by the last block alone, once every block has
    // summed the gradients (a block writing its own slice earlier would change what a slower block
    // reads for its norm)
    if (last_sh) {
      const int64_t tot_n = L.off[tb.n];
      const float cf = coef_sh;
      int jj = 0;
      int64_t lo = 0, hi = L.off[1];
      float* gp = L.g[0];
      for (int64_t q = threadIdx.x; q < tot_n; q += NTH) {
        while (q >= hi && jj + 1 < tb.n) {
          ++jj;
          lo = hi;
          hi = L.off[jj + 1];
          gp = L.g[jj];
        }
        gp[q - lo] = gp[q - lo] * cf;
      }
    }
  }
  const float coef = coef_sh;
  const double t = (double)(SELF ? snap_sh : partial[step_off]) + 1.0;
  const double bc1 = 1.0 - pow(beta1, t), bc2 = 1.0 - pow(beta2, t);
  const float neg_step = (float)(-lr / bc1), bc2s = (float)sqrt(bc2);
  const float b2 = (float)beta2, omb1 = (float)(1.0 - beta1), omb2 = (float)(1.0 - beta2);
  const float epsf = (float)eps, wdf = (float)wd;
  for (int64_t e = e0 + threadIdx.x; has && e < e1; e += kAdamUnroll * NTH) {
    if (e != e0 + threadIdx.x) load_pass(e);  // (the first pass was loaded before the reduction)
#pragma unroll
    for (int u = 0; u < kAdamUnroll; ++u) {
      if (!ok[u]) continue;
      float g = g0[u] * coef;
      if constexpr (!SELF) L.g[j[u]][i[u]] = g;  // clip_grad_norm_ scales .grad in place (SELF: above)
      if (wdf != 0.f) g = g + wdf * p[u];  // Adam (not AdamW) weight decay: grad.add(param, alpha=wd)
      const float m = fmaf(omb1, g - m0[u], m0[u]);  // exp_avg.lerp_(grad, 1 - beta1)
      const float v = v0[u] * b2 + omb2 * g * g;
      L.m[j[u]][i[u]] = m;
      L.v[j[u]][i[u]] = v;
      L.p[j[u]][i[u]] = p[u] + neg_step * (m / (sqrtf(v) / bc2s + epsf));
    }
  }
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_masked_ce_workspace_size(int64_t N, size_t* bytes) {
  if (!bytes || N < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  *bytes = (size_t)std::max<int64_t>(1, ceil_div(N, kCeThreads)) * sizeof(float);
  return GNN_OK;
}

extern "C" gnn_status gnn_masked_ce_f32(int64_t N, int32_t C, const float* logits, int64_t ldx, const int64_t* y,
                                        const uint8_t* mask, const float* class_w, float inv_denom, float* dlogits,
                                        int64_t ld_d, float* loss, void* workspace, size_t workspace_bytes,
                                        gnn_stream_t stream) {
  if (N < 0 || C < 1 || C > kMaxClasses || ldx < C || ld_d < C || (N > 0 && (!logits || !y || !mask ||
                                                                               !class_w || !dlogits)))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad args (1 <= C <= 16)");
  const int nblk = (int)std::max<int64_t>(1, ceil_div(N, kCeThreads));
  if (!workspace || workspace_bytes < nblk * sizeof(float)) return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* partial = static_cast<float*>(workspace);
  if (N == 0) {
    if (!loss) return hip_check(hipMemsetAsync(partial, 0, sizeof(float), st), __func__);  // one zero partial
    return hip_check(hipMemsetAsync(loss, 0, sizeof(float), st), __func__);
  }
  if (C == 2)
    masked_ce_kernel<2><<<nblk, kCeThreads, 0, st>>>(N, C, logits, ldx, y, mask, class_w, inv_denom, dlogits, ld_d,
                                                     partial);
  else
    masked_ce_kernel<0><<<nblk, kCeThreads, 0, st>>>(N, C, logits, ldx, y, mask, class_w, inv_denom, dlogits, ld_d,
                                                     partial);
  GNN_LAUNCH_CHECK();
  if (!loss) return GNN_OK;  // the partials stay in the workspace (gnn_masked_ce_finish / ClipAdam)
  sum_partials_kernel<<<1, 256, 0, st>>>(partial, nblk, inv_denom, loss);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_masked_ce_colsum_f32(int64_t N, int32_t C, const float* logits, int64_t ldx,
                                               const int64_t* y, const uint8_t* mask, const float* class_w,
                                               float inv_denom, float* dlogits, int64_t ld_d, float* loss,
                                               void* workspace, size_t workspace_bytes, float* colsum,
                                               gnn_stream_t stream) {
  if (N < 1 || C < 1 || C > kMaxClasses || ldx < C || ld_d < C || !logits || !y || !mask || !class_w ||
      !dlogits || !colsum)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad args (N >= 1, 1 <= C <= 16, colsum)");
  const int nblk = (int)ceil_div(N, kCeThreads);
  if (!workspace || workspace_bytes < nblk * sizeof(float)) return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* partial = static_cast<float*>(workspace);
  if (C == 2)
    masked_ce_kernel<2><<<nblk, kCeThreads, 0, st>>>(N, C, logits, ldx, y, mask, class_w, inv_denom, dlogits, ld_d,
                                                     partial, colsum);
  else
    masked_ce_kernel<0><<<nblk, kCeThreads, 0, st>>>(N, C, logits, ldx, y, mask, class_w, inv_denom, dlogits, ld_d,
                                                     partial, colsum);
  GNN_LAUNCH_CHECK();
  if (!loss) return GNN_OK;
  sum_partials_kernel<<<1, 256, 0, st>>>(partial, nblk, inv_denom, loss);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_masked_ce_finish(const float* partial, int32_t nblk, float inv_denom, float* loss,
                                           gnn_stream_t stream) {
  if (!partial || !loss || nblk < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  sum_partials_kernel<<<1, 256, 0, (hipStream_t)stream>>>(partial, nblk, inv_denom, loss);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

// workspace: the grad_sq partials (2 kAdamBlocks + 1 floats), then the SELF form's block counter
// (one word; zero before the first call, left zero by every call)
constexpr size_t kAdamWsBytes = (2 * kAdamBlocks + 2) * sizeof(float);
extern "C" gnn_status gnn_clip_adam_workspace_size(size_t* bytes) {
  if (!bytes) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  *bytes = kAdamWsBytes;
  return GNN_OK;
}

extern "C" gnn_status gnn_clip_adam_f32(const gnn_adam_group* grp, float* step, float* norm_out, void* workspace,
                                        size_t workspace_bytes, gnn_stream_t stream) {
  if (!grp || !step || grp->num_tensors < 0 || grp->num_tensors > GNN_ADAM_MAX_TENSORS)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad group");
  if (!workspace || workspace_bytes < kAdamWsBytes) return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  AdamTable tb{};
  tb.n = grp->num_tensors;
  tb.off[0] = 0;
  for (int j = 0; j < tb.n; ++j) {
    const gnn_adam_tensor& t = grp->tensors[j];
    if (t.numel < 0 || (t.numel > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq)))
      return fail(GNN_ERR_INVALID_ARG, __func__, "bad tensor");
    tb.p[j] = t.param; tb.g[j] = t.grad; tb.m[j] = t.exp_avg; tb.v[j] = t.exp_avg_sq;
    tb.off[j + 1] = tb.off[j] + t.numel;
  }
  hipStream_t st = (hipStream_t)stream;
  float* partial = static_cast<float*>(workspace);
  LossFinish lf{grp->loss_partial, grp->loss_nblk, grp->loss_scale, grp->loss_out};
  if (lf.partial && (!lf.out || lf.n < 1)) return fail(GNN_ERR_INVALID_ARG, __func__, "loss_partial needs loss_out and loss_nblk >= 1");
  if (grp->grad_sq_partial) {  // ABI 20: the norm partials came with the gradients (the TN's reduce)
    if (grp->grad_sq_nblk < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "grad_sq_partial needs grad_sq_nblk >= 1");
    const int nb = grp->grad_sq_nblk;
    clip_adam_kernel<<<kAdamBlocks + (lf.partial ? 1 : 0), kAdamThreads, 0, st>>>(tb, grp->grad_sq_partial, nb, nb, 2 * nb, step,
                                                           grp->max_norm, grp->lr, grp->beta1, grp->beta2, grp->eps,
                                                           grp->weight_decay, norm_out, grp->skip_nonfinite,
                                                           grp->bump_counter, lf);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  if (tb.off[tb.n] <= kSelfMax) {  // one launch: every block sums Σg² itself
    unsigned* done = reinterpret_cast<unsigned*>(partial + 2 * kAdamBlocks + 1);
    clip_adam_kernel<kSelfThreads, true><<<kAdamBlocks + (lf.partial ? 1 : 0), kSelfThreads, 0, st>>>(
        tb, partial, 0, 0, 0, step, grp->max_norm, grp->lr, grp->beta1, grp->beta2, grp->eps, grp->weight_decay,
        norm_out, grp->skip_nonfinite, grp->bump_counter, lf, done);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  grad_sq_kernel<<<kAdamBlocks, kAdamThreads, 0, st>>>(tb, partial, step, lf);
  GNN_LAUNCH_CHECK();
  clip_adam_kernel<<<kAdamBlocks, kAdamThreads, 0, st>>>(tb, partial, kAdamBlocks, kAdamBlocks + 1, kAdamBlocks, step,
                                                         grp->max_norm, grp->lr, grp->beta1, grp->beta2, grp->eps,
                                                         grp->weight_decay, norm_out, grp->skip_nonfinite,
                                                         grp->bump_counter, LossFinish{});
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
