// stride_probe — the gait composer's write pattern with different row strides: per problem a contiguous range of
// `rowlen` 16-byte units (the FDISC values, 1.47 MB) at the start of a row of `rowstride` units, written as
// block-contiguous chunks in the kernels' XCD-chunked work order, kGroup problems per block (gstream.hip
// towr_gait_compose_kernel's geometry: 512 threads, 32 chunks per problem, 2 problems per block). Prints GB/s of the
// bytes written. A measurement tool, not part of the product.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/build/stride_probe tools/stride_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl2_t __attribute__((ext_vector_type(2)));

// block w (XCD-chunked) = (problem group g, chunk j); writes chunk j of problems g, g + ng, ... (ng groups)
// mode 0: lane l of trip t stores unit c0 + 512 t + l (the composers); 1: the trips aligned to 1 KB of the row (unit
// (c0 & ~63) + 512 t + l, the units before c0 masked); 2: the chunk bounds rounded down to 1 KB (ideal)
__global__ void __launch_bounds__(512) compose_like(dbl2_t* p, int B, int ng, int nchunk, int rowlen, long rowstride, int mode) {
  const int per = (gridDim.x + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  const int g = w / nchunk, j = w - g * nchunk;
  if (g >= ng) return;
  int c0 = (int)((long)j * rowlen / nchunk), c1 = (int)((long)(j + 1) * rowlen / nchunk);
  if (mode == 2) { c0 &= ~63; if (j + 1 < nchunk) c1 &= ~63; }
  const int s0 = mode == 1 ? (c0 & ~63) : c0;
  for (int b = g; b < B; b += ng) {
    dbl2_t* row = p + (long)b * rowstride;
    for (int i = s0 + (int)threadIdx.x; i < c1; i += 512) {
      dbl2_t z = {(double)i, 1.0};
      if (i >= c0) __builtin_nontemporal_store(z, row + i);
    }
  }
}

int main() {
  const int B = 1024, nchunk = 32, rowlen = 1474000 / 16;   // ~1.47 MB per problem
  dbl2_t* a;
  const size_t bytes = (size_t)B * (4ull << 20);   // row strides up to 4 MB
  if (hipMalloc(&a, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, long rowstride, int ng, int mode = 0) {
    if ((size_t)(B - 1) * rowstride * 16 + (size_t)rowlen * 16 > bytes) { std::printf("%s: too large\n", name); return; }
    const unsigned grid = (unsigned)(((long)ng * nchunk + 7) / 8 * 8);
    for (int i = 0; i < 3; ++i) compose_like<<<grid, 512>>>(a, B, ng, nchunk, rowlen, rowstride, mode);
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) compose_like<<<grid, 512>>>(a, B, ng, nchunk, rowlen, rowstride, mode);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double by = (double)B * rowlen * 16;
    std::printf("%-52s %8.4f ms  %7.1f GB/s\n", name, ms / reps, by / (ms / reps * 1e-3) / 1e9);
  };
  char nm[128];
  const long real = 1930112 / 16;   // the bench's row: nnz rounded up to 16 doubles
  for (int ng : {B / 2, B})
    for (int mode : {1, 2}) {
      std::snprintf(nm, sizeof nm, "bench row stride, %d per block, %s", B / ng, mode == 1 ? "1 KB-aligned trips" : "1 KB chunk bounds");
      run(nm, real, ng, mode);
    }
  for (int ng : {B / 2, B}) {
    std::snprintf(nm, sizeof nm, "contiguous rows, %d problem(s) per block", B / ng);
    run(nm, rowlen, ng);
    std::snprintf(nm, sizeof nm, "bench row stride 1.93 MB, %d per block", B / ng);
    run(nm, real, ng);
    for (long s : {1536l << 10, 2l << 20, 2048l * 1024 + 4096, 3l << 20}) {
      std::snprintf(nm, sizeof nm, "row stride %ld KB, %d per block", s >> 10, B / ng);
      run(nm, s / 16, ng);
    }
    std::snprintf(nm, sizeof nm, "bench stride + 4 KB, %d per block", B / ng);
    run(nm, real + 256, ng);
    std::snprintf(nm, sizeof nm, "bench stride + 64 KB, %d per block", B / ng);
    run(nm, real + 4096, ng);
  }
  return 0;
}
