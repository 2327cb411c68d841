// Kernel lab (not part of the library): does a chain of dependent v_mfma_f32_32x32x16_f16 (one
// accumulator, as the half-pair NT's tile) issue slower than the same MFMAs over 2 / 4 independent
// accumulators?  One 256-thread block per CU (one wave per SIMD, the NT's occupancy), each wave runs
// ITER x 24 MFMAs; the operands are loop-invariant registers (no memory in the loop).  Run under
// rocprofv3 --kernel-trace --stats:  make -C elliptic_gnn_project_amd/csrc labmfma; ./lab_mfma
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_chain_kernel(float* out, int iters, float seed) {
  f16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(seed * (threadIdx.x + i));
    b[i] = (_Float16)(seed * (i - (int)threadIdx.x));
  }
  floatx16 acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 24; ++m) acc[m % NACC] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[m % NACC], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[q][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  float* out;
  if (hipMalloc(&out, 256 * 256 * sizeof(float)) != hipSuccess) return 1;
  for (int r = 0; r < 5; ++r) {
    mfma_chain_kernel<1><<<256, 256>>>(out, iters, 1e-3f);
    mfma_chain_kernel<2><<<256, 256>>>(out, iters, 1e-3f);
    mfma_chain_kernel<3><<<256, 256>>>(out, iters, 1e-3f);
    mfma_chain_kernel<4><<<256, 256>>>(out, iters, 1e-3f);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("iters %d x 24 MFMAs per wave: %.3f us at 32 cycles / MFMA and 2.4 GHz\n", iters,
              iters * 24 * 32 / 2400.0);
  return 0;
}
