// bw_probe2 — write-pattern ceilings for the streaming gait composer (towr2025_amd/csrc/fstream.hip):
// 16-byte non-temporal stores of zeros over 1.5 GB, as block-contiguous chunks in the kernels'
// XCD-chunked work order (chunk size, block size, stores in flight), grid-stride, and the real
// layout (per problem a 1.48 MB range inside a 1.93 MB row). Prints GB/s. Tool, not product.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl2_t __attribute__((ext_vector_type(2)));

template <int U>
__global__ void chunk_xcd(dbl2_t* p, size_t n, int chunk, int rowlen, int rowstride) {
  // chunk w (XCD-chunked order) -> units [w*chunk, (w+1)*chunk) of a virtual range; virtual unit v maps
  // to row v / rowlen, offset v % rowlen (rowlen == rowstride: contiguous)
  const int per = (gridDim.x + 7) / 8;
  const size_t w = (size_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  const size_t base = w * chunk;
  for (int i = threadIdx.x; i < chunk; i += U * blockDim.x) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t v = base + i + u * blockDim.x;
      if (i + u * (int)blockDim.x >= chunk || v >= n) break;
      const size_t a = (v / rowlen) * rowstride + v % rowlen;
      dbl2_t z = {0.0, 0.0};
      __builtin_nontemporal_store(z, p + a);
    }
  }
}
__global__ void gstride(dbl2_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    dbl2_t z = {0.0, 0.0};
    __builtin_nontemporal_store(z, p + i);
  }
}

int main() {
  const size_t bytes = 2000ull << 20, n = bytes / 16;
  dbl2_t* a;
  if (hipMalloc(&a, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch, double traffic) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::printf("%-44s %8.4f ms  %7.1f GB/s\n", name, ms / reps, traffic / (ms / reps * 1e-3) / 1e9);
  };
  const size_t nv = (size_t)1480 * 1024 * 1024 / 16;   // 1.48 GB of units
  for (int chunkKB : {192, 96, 48, 24, 12}) {
    for (int thr : {256, 512, 1024}) {
      const int chunk = chunkKB * 1024 / 16;
      const unsigned g = (unsigned)((nv + chunk - 1) / chunk);
      char nm[96];
      std::snprintf(nm, sizeof nm, "chunk %3d KB x%4d u1 contiguous", chunkKB, thr);
      run(nm, [&] { chunk_xcd<1><<<g, thr>>>(a, nv, chunk, chunk, chunk); }, nv * 16.0);
      std::snprintf(nm, sizeof nm, "chunk %3d KB x%4d u4 contiguous", chunkKB, thr);
      run(nm, [&] { chunk_xcd<4><<<g, thr>>>(a, nv, chunk, chunk, chunk); }, nv * 16.0);
    }
  }
  {   // the real gait layout: per problem 1.48 MB of FDISC inside a 1.93 MB row, 1024 problems
    const int rowlen = 1480 * 1024 / 16 * 1024 / 1000, rowstride = 1930 * 1024 / 16;
    for (int chunkKB : {192, 48}) {
      const int chunk = chunkKB * 1024 / 16;
      const size_t nr = (size_t)rowlen * 1000;
      const unsigned g = (unsigned)((nr + chunk - 1) / chunk);
      char nm[96];
      std::snprintf(nm, sizeof nm, "chunk %3d KB x256 u1 strided rows", chunkKB);
      run(nm, [&] { chunk_xcd<1><<<g, 256>>>(a, nr, chunk, rowlen, rowstride); }, nr * 16.0);
    }
  }
  for (int blocks : {256, 512, 1024, 2048, 8192, 16384}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "grid-stride %d x256", blocks);
    run(nm, [&] { gstride<<<blocks, 256>>>(a, nv); }, nv * 16.0);
  }
  run("hipMemsetAsync 1.48 GB", [&] { hipMemsetAsync(a, 0, nv * 16); }, nv * 16.0);
  return 0;
}
