// WRITE_SIZE calibration for the store widths the gait tile kernels use (measurement tool, not product):
// one launch per pattern over a 256 MB buffer, run under `rocprofv3 --kernel-trace --pmc WRITE_SIZE`.
//   wcal_store16: 16 B per lane, coalesced (the calibrated width, MI355X_MICROARCH.md HBM section)
//   wcal_store8:  8 B per lane, coalesced (the per-wave zero-fill loops)
//   wcal_sparse8: 8 B per lane, one double per 64-B line (scattered value stores), 1/8 of the bytes
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/build/wcal tools/wcal.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl2 __attribute__((ext_vector_type(2)));

__global__ void wcal_store16(dbl2* p, long n2) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) p[i] = dbl2{0.0, 0.0};
}
__global__ void wcal_store8(double* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = 0.0;
}
__global__ void wcal_sparse8(double* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i * 8 < n; i += (long)gridDim.x * blockDim.x) p[i * 8] = 1.0;
}

int main() {
  const long bytes = 256l << 20, n = bytes / 8;
  double* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) { std::printf("hipMalloc failed\n"); return 1; }
  for (int r = 0; r < 3; ++r) {
    wcal_store16<<<4096, 256>>>(reinterpret_cast<dbl2*>(p), n / 2);
    wcal_store8<<<4096, 256>>>(p, n);
    wcal_sparse8<<<4096, 256>>>(p, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) { std::printf("kernel failed\n"); return 1; }
  std::printf("bytes written: store16 %ld, store8 %ld, sparse8 %ld\n", bytes, bytes, bytes / 8);
  (void)hipFree(p);
  return 0;
}
