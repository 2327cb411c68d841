// Kernel lab (not part of the library): the half-pair NT / TN of the SAGE layer-1 shape at
// shard sizes (M = 27,196 / 52,466 / 102,957 / 203,769 rows: the largest shard of the 8 / 4 / 2 /
// 1-way timestep partition), with ablations and grid sizes, for the strong-scaling schedule.
// Run under rocprofv3 --kernel-trace --stats (every variant is its own template instance).
//   make -C elliptic_gnn_project_amd/csrc labsmall;  ./lab_small M [reps]
#define GNNMP_LAB 1
#include "../gemm_planes.hip"
#include "../gemm_ws.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

namespace gnnmp {
void set_last_error(const std::string&) {}
}

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

using namespace gnnmp;

__global__ void split_h2_kernel(const float* x, int64_t n2, uint16_t* img, int64_t ps) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n2) return;
  uint32_t h, l;
  split_h2_pair(x[2 * i], x[2 * i + 1], h, l);
  reinterpret_cast<uint32_t*>(img)[i] = h;
  reinterpret_cast<uint32_t*>(img + ps)[i] = l;
}

// the library's slab reduce (gemm_f32.hip), restated for the lab's timing
template <int NB>
__global__ __launch_bounds__(256) void lab_reduce_kernel(const float* __restrict__ slab, int64_t stride, int nblk,
                                                         float* __restrict__ out, int64_t n) {
  __shared__ float4 part[16][16];
  const int o = threadIdx.x & 15;
  const int g = threadIdx.x / 16;
  const int64_t j = ((int64_t)blockIdx.x * 16 + o) * 4;
  const int per = (nblk + 15) / 16;
  const int b0 = g * per, b1 = min(nblk, b0 + per);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < n)
    for (int b = b0; b < b1; ++b) {
      float4 v = *reinterpret_cast<const float4*>(slab + (int64_t)b * stride + j);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  part[g][o] = s;
  __syncthreads();
  if (g != 0) return;
  float4 t = part[0][o];
  for (int q = 1; q < 16; ++q) {
    float4 v = part[q][o];
    t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
  }
  if (j + 3 < n) *reinterpret_cast<float4*>(out + j) = t;
}

constexpr int EPIF = WS_BIAS | WS_RELU | WS_DROP | WS_PROJ;

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? std::atoll(argv[1]) : 27196;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const int64_t F = 166, LD = 336, NR = 128;
  std::vector<float> hx(M * LD, 0.f);
  {
    std::mt19937 g(1);
    std::normal_distribution<float> d(0.f, 1.f);
    for (int64_t r = 0; r < M; ++r)
      for (int c = 0; c < F; ++c) {
        hx[r * LD + c] = d(g) * 0.7f;
        hx[r * LD + 168 + c] = d(g);
      }
  }
  auto up = [](const std::vector<float>& h) {
    float* p;
    CK(hipMalloc(&p, h.size() * 4));
    CK(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return p;
  };
  float* xa = up(hx);
  uint16_t* imh;
  CK(hipMalloc(&imh, 2 * M * LD * 2));
  split_h2_kernel<<<(unsigned)ceil_div(M * LD / 2, 256), 256>>>(xa, M * LD / 2, imh, M * LD);
  std::vector<float> hw1(NR * F), hw2(NR * F), hb(NR), hp(4 * NR), hh(M * NR), hdz(M * 4);
  {
    std::mt19937 g(5);
    std::normal_distribution<float> d(0.f, 1.f);
    for (auto& v : hw1) v = d(g) * 0.08f;
    for (auto& v : hw2) v = d(g) * 0.08f;
    for (auto& v : hb) v = d(g) * 0.1f;
    for (auto& v : hp) v = d(g);
    for (auto& v : hh) v = d(g);
    for (auto& v : hdz) v = d(g) * 1e-5f;
  }
  float *w1 = up(hw1), *w2 = up(hw2), *bias = up(hb), *proj = up(hp), *dh = up(hh), *ddz = up(hdz);
  float *c, *z;
  CK(hipMalloc(&c, M * NR * 4));
  CK(hipMalloc(&z, M * 4 * 4));
  NTArgs n{};
  n.M = M; n.Nc = NR; n.k1 = F; n.k2 = F; n.w1 = w1; n.w2 = w2; n.ldw1 = F; n.ldw2 = F; n.c = c; n.ldc = NR;
  n.bias = bias; n.relu = 1; n.dropout = 1; n.keep_thresh = (uint32_t)(0.5 * 16777216.0); n.drop_scale = 2.f;
  n.seed = 1234; n.proj = proj; n.nproj = 4; n.z = z; n.ldz = 4;
  n.ap = imh; n.ap_ld = LD; n.ap_col2 = 168; n.ap_ps = M * LD; n.ap_h2 = 1;
  uint4* bh;
  CK(hipMalloc(&bh, 21 * 3 * 256 * 16 + 128 * 4));
  float* cs = reinterpret_cast<float*>(bh + 21 * 3 * 256);
  ws_prep_h2_kernel<<<WS_PREP_GRID, WS_PREP_THREADS>>>(h2_prep_of(n, bh));
  const int ntiles = (int)ceil_div(M, 32);

  const int64_t stride = (NR * 332 + NR + 4 * NR + 4 + 63) / 64 * 64;
  float *slab, *out;
  CK(hipMalloc(&slab, 256 * stride * 4));
  CK(hipMalloc(&out, stride * 4));
  TNArgs ta{};
  ta.M = M; ta.Nr = NR; ta.dz = ddz; ta.lddz = 4; ta.proj = proj; ta.nproj = 4; ta.h = dh; ta.ldh = NR; ta.hscale = 2.f;
  ta.k1 = F; ta.k2 = F; ta.slab = slab; ta.slab_stride = stride;
  ta.ap = imh; ta.ap_ld = LD; ta.ap_col2 = 168; ta.ap_ps = M * LD; ta.ap_h2 = 1;
  auto tn_args = [&](int nblk) {
    TNArgs t = ta;
    t.rows_per_block = ceil_div(ceil_div(M, 32), nblk) * 32;
    return t;
  };
  const int nout = (int)(NR * 332 + NR + 4 * NR + 4);
  const unsigned rb = (unsigned)ceil_div(ceil_div(nout, 4), 16);
  for (int r = 0; r < reps; ++r) {
    gemm_nt_h2_kernel<21, EPIF, 0><<<std::min(ntiles, 256), 256>>>(n, bh, cs, ntiles);
    gemm_nt_h2_kernel<21, EPIF, 1><<<std::min(ntiles, 256), 256>>>(n, bh, cs, ntiles);  // no MFMA
    gemm_nt_h2_kernel<21, EPIF, 2><<<std::min(ntiles, 256), 256>>>(n, bh, cs, ntiles);  // no epilogue
    gemm_nt_h2_kernel<21, EPIF, 4><<<std::min(ntiles, 256), 256>>>(n, bh, cs, ntiles);  // no staging
    gemm_nt_h2_kernel<21, EPIF, 6><<<std::min(ntiles, 256), 256>>>(n, bh, cs, ntiles);  // MFMA only
    gemm_nt_h2_kernel<21, EPIF, 7><<<std::min(ntiles, 256), 256>>>(n, bh, cs, ntiles);  // B load + frame only
    gemm_nt_h2_kernel<21, EPIF | 64, 0><<<std::min(ntiles, 128), 256>>>(n, bh, cs, ntiles);  // 128 blocks (tag 64)
    for (int nb : {std::min(256, (int)ceil_div(ceil_div(M, 32), ceil_div(ceil_div(M, 32), 256))), 128, 64}) {
      TNArgs t = tn_args(nb);
      if (nb > 128) {
        gemm_tn_h2_kernel<11, false, 0, 8><<<nb, 512>>>(t);
        gemm_tn_h2_kernel<11, false, 1, 8><<<nb, 512>>>(t);  // no MFMA
        gemm_tn_h2_kernel<11, false, 2, 8><<<nb, 512>>>(t);  // no staging
        gemm_tn_h2_kernel<11, false, 128, 8><<<nb, 512>>>(t);  // no slab stores
        gemm_tn_h2_kernel<11, false, 3, 8><<<nb, 512>>>(t);  // no MFMA, no staging: prologue + slab
        gemm_tn_h2_kernel<11, false, 131, 8><<<nb, 512>>>(t);  // prologue only
        gemm_tn_h2_kernel<11, false, 16, 8><<<nb, 512>>>(t);  // A ring of two sets (3 chunks ahead)
        lab_reduce_kernel<256><<<rb, 256>>>(slab, stride, nb, out, nout);
      } else if (nb == 128) {
        gemm_tn_h2_kernel<11, false, 32, 8><<<nb, 512>>>(t);  // (tag 32: the same kernel at 128 blocks)
        lab_reduce_kernel<128><<<rb, 256>>>(slab, stride, nb, out, nout);
      } else {
        gemm_tn_h2_kernel<11, false, 64, 8><<<nb, 512>>>(t);  // (tag 64: 64 blocks)
        lab_reduce_kernel<64><<<rb, 256>>>(slab, stride, nb, out, nout);
      }
    }
  }
  CK(hipDeviceSynchronize());
  std::printf("M %lld ntiles %d done\n", (long long)M, ntiles);
  return 0;
}
