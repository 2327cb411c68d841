// Shared helpers for libgnnmp (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/gnnmp.h"

namespace gnnmp {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

void set_last_error(const std::string& msg);

inline gnn_status fail(gnn_status s, const char* fn, const char* what) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", fn, what);
  set_last_error(buf);
  return s;
}

inline gnn_status hip_check(hipError_t e, const char* fn) {
  if (e == hipSuccess) return GNN_OK;
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: HIP error %d (%s)", fn, static_cast<int>(e),
                hipGetErrorString(e));
  set_last_error(buf);
  return GNN_ERR_HIP;
}

#define GNN_HIP_TRY(expr)                                 \
  do {                                                    \
    gnn_status _s = ::gnnmp::hip_check((expr), __func__); \
    if (_s != GNN_OK) return _s;                          \
  } while (0)

#define GNN_LAUNCH_CHECK() GNN_HIP_TRY(hipGetLastError())

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace (256-B aligned carves).
struct WorkspaceCarver {
  char* base;
  size_t cap;
  size_t used = 0;
  bool ok = true;
  WorkspaceCarver(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    size_t off = align_up(used, 256);
    size_t bytes = align_up(count * sizeof(T), 256);
    if (off + bytes > cap) {
      ok = false;
      return nullptr;
    }
    used = off + bytes;
    return reinterpret_cast<T*>(base + off);
  }
};

// Sizes-only twin of WorkspaceCarver (same carve rules).
struct WorkspaceSizer {
  size_t used = 0;
  template <typename T>
  void take(size_t count) {
    used = align_up(used, 256) + align_up(count * sizeof(T), 256);
  }
};

// One row of the masked weighted cross entropy (F.cross_entropy(weight=w, reduction='none'),
// src/train_gnn.py:159-175) and its gradient: v[0..C) the row's logits (overwritten with exp(v - max)),
// returns loss = -wt·log_softmax(v)[t] when ``on``, writes dl[c] = wt·inv·(softmax - onehot) (0 when
// off).  Shared by train_ops.hip's masked_ce_kernel and aggregate.hip's fused output mean + CE,
// which build with different -ffp-contract settings: contraction is off here (and the one FMA is
// written out), so both produce the same bits.
// expf / logf as ROCm's device library computes them (extended-precision range reduction around
// v_exp_f32 / v_log_f32), every operation written out: the library's own fmul + fadd pairs are
// contracted or not depending on the including file's -ffp-contract, which moved a row's loss by
// one ulp between the two kernels below.
__device__ __forceinline__ float ce_expf(float x) {
#pragma clang fp contract(off)
  const float l2e = __uint_as_float(0x3fb8aa3bu), l2e_lo = __uint_as_float(0x32a5705fu);
  const float ph = x * l2e;
  float pl = fmaf(x, l2e, -ph);
  pl = fmaf(x, l2e_lo, pl);
  const float e = __builtin_rintf(ph);
  const float t = (ph - e) + pl;
  float r = __builtin_ldexpf(__builtin_amdgcn_exp2f(t), (int)e);
  r = x < __uint_as_float(0xc2ce8ed0u) ? 0.f : r;         // below -103.97: 0
  r = x > __uint_as_float(0x42b17218u) ? __uint_as_float(0x7f800000u) : r;  // above 88.72: inf
  return r;
}

__device__ __forceinline__ float ce_logf(float x) {
#pragma clang fp contract(off)
  const float ln2 = __uint_as_float(0x3f317217u), ln2_lo = __uint_as_float(0x3377d1cfu);
  const bool tiny = x < __uint_as_float(0x00800000u);  // subnormal: scaled by 2^32 first
  const float y = __builtin_amdgcn_logf(tiny ? __builtin_ldexpf(x, 32) : x);  // log2
  const float r = y * ln2;
  float e = fmaf(y, ln2, -r);
  e = fmaf(y, ln2_lo, e);
  const float v = fabsf(y) < __uint_as_float(0x7f800000u) ? r + e : y;
  return v - (tiny ? __uint_as_float(0x41b17218u) : 0.f);  // 32·ln2
}

template <int CM>
__device__ __forceinline__ float masked_ce_row(float (&v)[CM], int C, int64_t t, bool on, float wt, float inv,
                                               float* __restrict__ dl, float* dlv = nullptr) {
#pragma clang fp contract(off)
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) mx = fmaxf(mx, v[c]);
  float s = 0.f, xt = 0.f;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      if (c == t) xt = v[c];
      v[c] = ce_expf(v[c] - mx);
      s += v[c];
    }
  const float l = on ? -wt * (xt - mx - ce_logf(s)) : 0.f;
  const float g = wt * inv, rs = 1.0f / s;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      const float d = on ? g * fmaf(v[c], rs, c == t ? -1.f : 0.f) : 0.f;
      dl[c] = d;
      if (dlv) dlv[c] = d;  // (the caller's copy: aggregate.hip's per-row term of the transposed mean)
    }
  return l;
}

}  // namespace gnnmp
