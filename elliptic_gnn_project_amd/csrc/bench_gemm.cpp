// Kernel lab: times libgnnmp GEMM kernels through the C ABI on the Elliptic SAGE-preset shapes
// (hipEvent timing, variants interleaved in one process, median of rounds) and checks every
// variant against a float64 host reference.
//   ./bench_gemm [M] [rounds]
// Not part of the library; built by `make lab`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/gnnmp.h"

extern "C" gnn_status gnnx_gemm_nt_variant_f32(const gnn_gemm_nt_params* p, int variant, gnn_stream_t stream);
extern "C" gnn_status gnnx_gemm_tn_variant_f32(const gnn_gemm_tn_params* p, float* out, void* workspace,
                                               size_t workspace_bytes, int variant, gnn_stream_t stream);

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)
#define GK(x)                                                                  \
  do {                                                                         \
    gnn_status s = (x);                                                        \
    if (s != GNN_OK) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, gnn_status_string(s), gnn_last_error()); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

static std::vector<float> host_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::normal_distribution<float> d(0.f, scale);
  for (auto& v : h) v = d(g);
  return h;
}
static float* to_dev(const std::vector<float>& h) {
  float* p;
  CK(hipMalloc(&p, h.size() * sizeof(float)));
  CK(hipMemcpy(p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  return p;
}
static std::vector<float> to_host(const float* d, size_t n) {
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), d, n * sizeof(float), hipMemcpyDeviceToHost));
  return h;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  template <typename F>
  float run(F f, int reps) {
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
  }
};
static float med(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? std::atoll(argv[1]) : 203769;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 7;
  const int64_t F = std::getenv("LAB_F") ? std::atoll(std::getenv("LAB_F")) : 166, H = 128;
  // LAB_PAD: rows stored with a 16-byte pitch (ld = F rounded up to 4), pad columns NaN (must be ignored)
  const int64_t LD = std::getenv("LAB_PAD") ? (F + 3) / 4 * 4 : F;
  auto h_agg = host_rand(M * F, 1.f, 1), h_x = host_rand(M * F, 1.f, 2);
  auto h_w = host_rand(2 * F * H, 0.08f, 7), h_bias = host_rand(H, 0.1f, 4), h_proj = host_rand(4 * H, 0.1f, 5);
  auto h_dz = host_rand(M * 4, 1e-3f, 6);
  auto pad = [&](const std::vector<float>& v) {
    std::vector<float> o(M * LD, std::nanf(""));
    for (int64_t r = 0; r < M; ++r) std::copy(v.begin() + r * F, v.begin() + (r + 1) * F, o.begin() + r * LD);
    return o;
  };
  float *agg = to_dev(LD == F ? h_agg : pad(h_agg)), *x = to_dev(LD == F ? h_x : pad(h_x));
  float *w = to_dev(h_w), *bias = to_dev(h_bias), *proj = to_dev(h_proj);
  float* dz = to_dev(h_dz);
  float *c, *z;
  CK(hipMalloc(&c, M * H * sizeof(float)));
  CK(hipMalloc(&z, M * 4 * sizeof(float)));

  gnn_gemm_nt_params p{};
  p.M = M; p.N = H;
  p.a1 = agg; p.lda1 = LD; p.k1 = F;
  p.a2 = x; p.lda2 = LD; p.k2 = F;
  p.w1 = w; p.w2 = w + F * H; p.ldw1 = F; p.ldw2 = F;
  p.c = c; p.ldc = H; p.bias = bias; p.relu = 1; p.dropout_p = 0.5f; p.seed = 1234;
  p.proj = proj; p.nproj = 4; p.z = z; p.ldz = 4;
  size_t ntws = 0;
  GK(gnn_gemm_nt_workspace_size(H, F, F, &ntws));
  CK(hipMalloc(&p.workspace, ntws));
  p.workspace_bytes = ntws;
  if (std::getenv("LAB_NOPROJ")) { p.proj = nullptr; p.nproj = 0; p.z = nullptr; }
  if (std::getenv("LAB_NODROP")) p.dropout_p = 0.f;
  gnn_gemm_nt_params plain = p;
  plain.bias = nullptr; plain.relu = 0; plain.dropout_p = 0.f; plain.proj = nullptr; plain.nproj = 0; plain.z = nullptr;

  if (const char* tn = std::getenv("LAB_TN_ONLY")) {  // one TN variant only (PMC passes): 0 = x3, 2 = x3b
    GK(gnnx_gemm_nt_variant_f32(&p, 16, nullptr));
    gnn_gemm_tn_params q{};
    q.M = M; q.Nr = H; q.dz = dz; q.lddz = 4; q.proj = proj; q.nproj = 4; q.h = c; q.ldh = H; q.hscale = 2.f;
    q.a1 = agg; q.lda1 = LD; q.k1 = F; q.a2 = x; q.lda2 = LD; q.k2 = F;
    size_t wsb = 0;
    GK(gnn_gemm_tn_workspace_size(M, H, 2 * F, 4, &wsb));
    void* ws;
    CK(hipMalloc(&ws, wsb));
    float* out;
    CK(hipMalloc(&out, (H * 2 * F + H + 4 * H + 4) * sizeof(float)));
    for (int r = 0; r < rounds; ++r) GK(gnnx_gemm_tn_variant_f32(&q, out, ws, wsb, std::atoi(tn), nullptr));
    CK(hipDeviceSynchronize());
    std::printf("LAB_TN_ONLY %s done\n", tn);
    return 0;
  }
  // ---- NT accuracy vs float64 on sampled rows (plain GEMM)
  std::vector<int> variants = {0, 1, 2, 16};  // 0 production, 1/2 pipelined orders, >=16: exact f32
  if (const char* vs = std::getenv("LAB_NT_VARIANTS")) {  // e.g. "0,6,7,8,9"
    variants.clear();
    for (const char* q = vs; *q;) {
      variants.push_back(std::atoi(q));
      while (*q && *q != ',') ++q;
      if (*q == ',') ++q;
    }
  }
  std::vector<int64_t> rows;
  for (int64_t r = 0; r < M; r += std::max<int64_t>(1, M / 3000)) rows.push_back(r);
  rows.push_back(M - 1);
  std::vector<double> ref(rows.size() * H);
  double refmax = 0.0;
  for (size_t i = 0; i < rows.size(); ++i)
    for (int n = 0; n < H; ++n) {
      double s = 0.0;
      for (int k = 0; k < F; ++k) s += (double)h_agg[rows[i] * F + k] * h_w[n * F + k];
      for (int k = 0; k < F; ++k) s += (double)h_x[rows[i] * F + k] * h_w[F * H + n * F + k];
      ref[i * H + n] = s;
      refmax = std::max(refmax, std::fabs(s));
    }
  for (int v : variants) {
    GK(gnnx_gemm_nt_variant_f32(&plain, v, nullptr));
    auto got = to_host(c, M * H);
    double maxabs = 0.0, maxrel = 0.0, se = 0.0, sr = 0.0;
    for (size_t i = 0; i < rows.size(); ++i)
      for (int n = 0; n < H; ++n) {
        const double r = ref[i * H + n], d = std::fabs((double)got[rows[i] * H + n] - r);
        maxabs = std::max(maxabs, d);
        maxrel = std::max(maxrel, d / (1e-5 + std::fabs(r)));
        se += d * d; sr += r * r;
      }
    std::printf("NT variant %2d vs f64: max|err| %.3e (max|ref| %.2f)  max rel(1e-5 floor) %.3e  relL2 %.3e\n", v, maxabs,
                refmax, maxrel, std::sqrt(se / sr));
  }
  if (const char* only = std::getenv("LAB_ONLY")) {  // one variant, for rocprofv3 --pmc passes
    const int v = std::atoi(only);
    for (int r = 0; r < rounds; ++r) GK(gnnx_gemm_nt_variant_f32(&p, v, nullptr));
    CK(hipDeviceSynchronize());
    std::printf("LAB_ONLY %s done\n", only);
    return 0;
  }
  const double flops = 2.0 * M * (2 * F) * H;
  Timer T;
  // rounds interleave the variants (after one untimed warm-up pass), so clock ramp and thermal
  // drift do not favour whichever variant is measured last
  std::vector<std::vector<float>> te(variants.size()), tp(variants.size());
  for (int v : variants) {
    T.run([&] { gnnx_gemm_nt_variant_f32(&p, v, nullptr); }, 5);
    T.run([&] { gnnx_gemm_nt_variant_f32(&plain, v, nullptr); }, 5);
  }
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < variants.size(); ++i) {
      te[i].push_back(T.run([&] { gnnx_gemm_nt_variant_f32(&p, variants[i], nullptr); }, 5));
      tp[i].push_back(T.run([&] { gnnx_gemm_nt_variant_f32(&plain, variants[i], nullptr); }, 5));
    }
  for (size_t i = 0; i < variants.size(); ++i)
    std::printf("NT variant %2d: fused-epilogue %8.1f us (%6.1f TF)   plain %8.1f us (%6.1f TF)\n", variants[i],
                med(te[i]), flops / med(te[i]) * 1e-6, med(tp[i]), flops / med(tp[i]) * 1e-6);

  // ---- TN (dz form + mask), the backward weight-gradient shape.  h = NT output (fused epilogue).
  GK(gnnx_gemm_nt_variant_f32(&p, 16, nullptr));
  gnn_gemm_tn_params q{};
  q.M = M; q.Nr = H; q.dz = dz; q.lddz = 4; q.proj = proj; q.nproj = 4; q.h = c; q.ldh = H; q.hscale = 2.f;
  q.a1 = agg; q.lda1 = LD; q.k1 = F; q.a2 = x; q.lda2 = LD; q.k2 = F;
  size_t wsb = 0;
  GK(gnn_gemm_tn_workspace_size(M, H, 2 * F, 4, &wsb));
  void* ws;
  CK(hipMalloc(&ws, wsb));
  const int64_t nout = H * 2 * F + H + 4 * H + 4;
  float* out;
  CK(hipMalloc(&out, nout * sizeof(float)));
  {  // accuracy on the first Mc rows (float64 host reference)
    const int64_t Mc = std::min<int64_t>(M, 20000);
    gnn_gemm_tn_params qc = q;
    qc.M = Mc;
    auto h_h = to_host(c, Mc * H);
    std::vector<double> rdw(H * 2 * F, 0.0), rdb(H, 0.0);
    std::vector<double> g(H);
    for (int64_t m = 0; m < Mc; ++m) {
      for (int n = 0; n < H; ++n) {
        double s = 0.0;
        for (int qq = 0; qq < 4; ++qq) s += (double)h_dz[m * 4 + qq] * h_proj[qq * H + n];
        // the kernels form G in f32 (fmaf chain), so compare on the same f32 G
        float gf = h_dz[m * 4 + 0] * h_proj[n];
        for (int qq = 1; qq < 4; ++qq) gf = std::fma(h_dz[m * 4 + qq], h_proj[qq * H + n], gf);
        gf = h_h[m * H + n] > 0.f ? gf * 2.f : 0.f;
        g[n] = gf;
        rdb[n] += gf;
        (void)s;
      }
      for (int n = 0; n < H; ++n) {
        if (g[n] == 0.0) continue;
        for (int k = 0; k < F; ++k) rdw[n * F + k] += g[n] * h_agg[m * F + k];
        for (int k = 0; k < F; ++k) rdw[H * F + n * F + k] += g[n] * h_x[m * F + k];
      }
    }
    for (int math : {1, 0, 3}) {  // 1: exact f32; 0: split-bf16 (production); 3: pipelined order
      qc.math = math >= 2 ? 0 : math;
      GK(gnnx_gemm_tn_variant_f32(&qc, out, ws, wsb, math >= 2 ? math : 0, nullptr));
      auto got = to_host(out, nout);
      double se = 0, sr = 0, mx = 0, rmx = 0;
      for (int64_t i = 0; i < H * 2 * F; ++i) {
        const double d = std::fabs(got[i] - rdw[i]);
        se += d * d; sr += rdw[i] * rdw[i]; mx = std::max(mx, d); rmx = std::max(rmx, std::fabs(rdw[i]));
      }
      double dbe = 0;
      for (int n = 0; n < H; ++n) dbe = std::max(dbe, std::fabs(got[H * 2 * F + n] - rdb[n]));
      std::printf("TN math=%d (M=%lld) vs f64: dW relL2 %.3e  max|err| %.3e (max|ref| %.3e)  db max|err| %.3e\n", math,
                  (long long)Mc, std::sqrt(se / sr), mx, rmx, dbe);
    }
  }
  std::vector<int> tmaths = {1, 0, 3, 4};  // 1 exact f32, 0 production, >= 2 lab variants
  if (const char* q = std::getenv("LAB_TN_VARIANTS")) {
    tmaths.clear();
    for (const char* t = q; *t;) { tmaths.push_back(std::atoi(t)); while (*t && *t != ',') ++t; if (*t) ++t; }
  }
  std::vector<std::vector<float>> tt(tmaths.size());
  auto tn_run = [&](int math) {
    q.math = math >= 2 ? 0 : math;
    return T.run([&] { gnnx_gemm_tn_variant_f32(&q, out, ws, wsb, math >= 2 ? math : 0, nullptr); }, 5);
  };
  for (int m : tmaths) tn_run(m);  // warm-up
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < tmaths.size(); ++i) tt[i].push_back(tn_run(tmaths[i]));
  for (size_t i = 0; i < tmaths.size(); ++i)
    std::printf("TN dz+mask math=%d: %8.1f us (%6.1f TF)\n", tmaths[i], med(tt[i]), flops / med(tt[i]) * 1e-6);
  return 0;
}
