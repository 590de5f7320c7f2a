// bw_probe — practical HBM ceilings on this MI355X for the engine's access pattern: streaming
// 16-byte writes (plain and non-temporal), streaming reads, and a copy, over 460 MB (the
// force_discretized launch's output at B = 4096). Prints GB/s per pattern. Tool, not product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double dbl2_t __attribute__((ext_vector_type(2)));

__global__ void w_nt(dbl2_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    dbl2_t v; v.x = (double)i; v.y = 1.0;
    __builtin_nontemporal_store(v, p + i);
  }
}
__global__ void w_plain(dbl2_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    dbl2_t v; v.x = (double)i; v.y = 1.0;
    p[i] = v;
  }
}
// block-contiguous chunks (like one tile per block): each block writes `chunk` consecutive units
__global__ void w_nt_chunk(dbl2_t* p, size_t n, int chunk) {
  const size_t base = (size_t)blockIdx.x * chunk;
  for (int i = threadIdx.x; i < chunk; i += blockDim.x) {
    if (base + i >= n) return;
    dbl2_t v; v.x = (double)i; v.y = 1.0;
    __builtin_nontemporal_store(v, p + base + i);
  }
}
// each lane stores U consecutive 16-B units (a wave covers 64*U*16 B contiguous)
template <int U>
__global__ void w_nt_u(dbl2_t* p, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i + U <= n; i += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) { dbl2_t v; v.x = (double)(i + u); v.y = 1.0; __builtin_nontemporal_store(v, p + i + u); }
  }
}
// wave-contiguous: lane l of a wave stores units base + u*64 + l (U stores of 1 KiB each)
template <int U>
__global__ void w_nt_wu(dbl2_t* p, size_t n) {
  const size_t waves = (size_t)gridDim.x * blockDim.x / 64, wid = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const int l = threadIdx.x & 63;
  for (size_t base = wid * 64 * U; base + 64 * U <= n; base += waves * 64 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) { dbl2_t v; v.x = (double)u; v.y = 1.0; __builtin_nontemporal_store(v, p + base + u * 64 + l); }
  }
}
// tile pattern with explicit cache-policy bits on global_store_dwordx4
template <int POL>
__global__ void w_tile_pol(dbl2_t* p, size_t n, int chunk) {
  const size_t base = (size_t)blockIdx.x * chunk;
  for (int i = threadIdx.x; i < chunk; i += blockDim.x) {
    if (base + i >= n) return;
    dbl2_t v; v.x = (double)i; v.y = 1.0;
    dbl2_t* q = p + base + i;
    if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off" :: "v"(q), "v"(v) : "memory");
    if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" :: "v"(q), "v"(v) : "memory");
    if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" :: "v"(q), "v"(v) : "memory");
    if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" :: "v"(q), "v"(v) : "memory");
    if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(q), "v"(v) : "memory");
    if constexpr (POL == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(q), "v"(v) : "memory");
  }
}
__global__ void r_sum(const dbl2_t* p, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    dbl2_t v = p[i]; s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
__global__ void copy_nt(const dbl2_t* a, dbl2_t* b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(a[i], b + i);
}

// wave-contiguous stores, U independent 1-KiB stores per wave in flight per iteration, grid-stride
template <int U>
__global__ void w_nt_wave_unroll(dbl2_t* p, size_t n) {
  const size_t nthr = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + (U - 1) * nthr < n; i += U * nthr) {
#pragma unroll
    for (int u = 0; u < U; ++u) { dbl2_t v; v.x = (double)u; v.y = 1.0; __builtin_nontemporal_store(v, p + i + u * nthr); }
  }
}
// block-contiguous chunk, U stores in flight per thread (stride blockDim)
template <int U>
__global__ void w_nt_chunk_u(dbl2_t* p, size_t n, int chunk) {
  const size_t base = (size_t)blockIdx.x * chunk;
  for (int i = threadIdx.x; i < chunk; i += U * blockDim.x) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = i + u * blockDim.x;
      if (k < chunk && base + k < n) { dbl2_t v; v.x = (double)k; v.y = 1.0; __builtin_nontemporal_store(v, p + base + k); }
    }
  }
}

// tile pattern with the engine's XCD-chunked work order: tile w = (blockIdx % 8) * per + blockIdx / 8
__global__ void w_nt_chunk_xcd(dbl2_t* p, size_t n, int chunk) {
  const int per = (gridDim.x + 7) / 8;
  const size_t w = (size_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  const size_t base = w * chunk;
  for (int i = threadIdx.x; i < chunk; i += blockDim.x) {
    if (base + i >= n) return;
    dbl2_t v; v.x = (double)i; v.y = 1.0;
    __builtin_nontemporal_store(v, p + base + i);
  }
}
// persistent tiles: gridDim blocks loop over tiles blockIdx, blockIdx + gridDim, ...
__global__ void w_nt_chunk_persist(dbl2_t* p, size_t n, int chunk, int ntiles) {
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t base = (size_t)t * chunk;
    for (int i = threadIdx.x; i < chunk; i += blockDim.x) {
      if (base + i >= n) break;
      dbl2_t v; v.x = (double)i; v.y = 1.0;
      __builtin_nontemporal_store(v, p + base + i);
    }
  }
}

int main() {
  const size_t bytes = 460ull << 20, n = bytes / 16;
  dbl2_t *a, *b; double* o;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&o, 8) != hipSuccess) return 1;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch, double traffic) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms / reps, traffic / (ms / reps * 1e-3) / 1e9);
  };
  for (int blocks : {1024, 2048, 4096, 16384}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "write_nt grid %d", blocks);
    run(nm, [&] { w_nt<<<blocks, 256>>>(a, n); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "write_plain grid %d", blocks);
    run(nm, [&] { w_plain<<<blocks, 256>>>(a, n); }, (double)bytes);
  }
  for (int chunk : {2300, 4600}) {   // ~37 KB / ~74 KB tiles
    char nm[64];
    std::snprintf(nm, sizeof nm, "write_nt tiles %d B", chunk * 16);
    run(nm, [&] { w_nt_chunk<<<(unsigned)((n + chunk - 1) / chunk), 192>>>(a, n, chunk); }, (double)bytes);
  }
  for (int blocks : {2048, 8192}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "write_nt_u4 grid %d", blocks);
    run(nm, [&] { w_nt_u<4><<<blocks, 256>>>(a, n); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "write_nt_wu4 grid %d", blocks);
    run(nm, [&] { w_nt_wu<4><<<blocks, 256>>>(a, n); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "write_nt_wu8 grid %d", blocks);
    run(nm, [&] { w_nt_wu<8><<<blocks, 256>>>(a, n); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "write_nt 1024thr grid %d", blocks / 4);
    run(nm, [&] { w_nt<<<blocks / 4, 1024>>>(a, n); }, (double)bytes);
  }
  {
    const int chunk = 2300;
    const unsigned g = (unsigned)((n + chunk - 1) / chunk);
    run("tile pol plain", [&] { w_tile_pol<0><<<g, 192>>>(a, n, chunk); }, (double)bytes);
    run("tile pol nt", [&] { w_tile_pol<1><<<g, 192>>>(a, n, chunk); }, (double)bytes);
    run("tile pol sc1 nt", [&] { w_tile_pol<2><<<g, 192>>>(a, n, chunk); }, (double)bytes);
    run("tile pol sc0 sc1 nt", [&] { w_tile_pol<3><<<g, 192>>>(a, n, chunk); }, (double)bytes);
    run("tile pol sc0 sc1", [&] { w_tile_pol<4><<<g, 192>>>(a, n, chunk); }, (double)bytes);
    run("tile pol sc1", [&] { w_tile_pol<5><<<g, 192>>>(a, n, chunk); }, (double)bytes);
  }
  for (int blocks : {1024, 2048, 4096}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "wave_unroll4 grid %d x256", blocks);
    run(nm, [&] { w_nt_wave_unroll<4><<<blocks, 256>>>(a, n); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "wave_unroll4 grid %d x1024", blocks / 4);
    run(nm, [&] { w_nt_wave_unroll<4><<<blocks / 4, 1024>>>(a, n); }, (double)bytes);
  }
  for (int chunk : {2300, 4600, 9200}) {
    char nm[64];
    const unsigned g = (unsigned)((n + chunk - 1) / chunk);
    std::snprintf(nm, sizeof nm, "chunk_u4 %d B x192", chunk * 16);
    run(nm, [&] { w_nt_chunk_u<4><<<g, 192>>>(a, n, chunk); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "chunk_u4 %d B x256", chunk * 16);
    run(nm, [&] { w_nt_chunk_u<4><<<g, 256>>>(a, n, chunk); }, (double)bytes);
    std::snprintf(nm, sizeof nm, "chunk_u1 %d B x512", chunk * 16);
    run(nm, [&] { w_nt_chunk_u<1><<<g, 512>>>(a, n, chunk); }, (double)bytes);
  }
  for (int blocks : {256, 512}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "write_nt grid %d", blocks);
    run(nm, [&] { w_nt<<<blocks, 256>>>(a, n); }, (double)bytes);
  }
  {
    const int chunk = 2300;
    const unsigned g = (unsigned)((n + chunk - 1) / chunk);
    run("tiles 36800 B xcd order", [&] { w_nt_chunk_xcd<<<g, 192>>>(a, n, chunk); }, (double)bytes);
    for (int pb : {256, 512, 768, 1024}) {
      char nm[64];
      std::snprintf(nm, sizeof nm, "tiles persistent %d x192", pb);
      run(nm, [&] { w_nt_chunk_persist<<<pb, 192>>>(a, n, chunk, (int)g); }, (double)bytes);
      std::snprintf(nm, sizeof nm, "tiles persistent %d x256", pb);
      run(nm, [&] { w_nt_chunk_persist<<<pb, 256>>>(a, n, chunk, (int)g); }, (double)bytes);
    }
  }
  run("read grid 4096", [&] { r_sum<<<4096, 256>>>(a, n, o); }, (double)bytes);
  run("copy_nt grid 4096", [&] { copy_nt<<<4096, 256>>>(a, b, n); }, 2.0 * bytes);
  run("hipMemsetAsync", [&] { hipMemsetAsync(a, 0, bytes); }, (double)bytes);
  run("hipMemsetD32Async", [&] { hipMemsetD32Async((hipDeviceptr_t)a, 0x3f800000, bytes / 4); }, (double)bytes);
  run("hipMemcpyAsync DtoD", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice); }, 2.0 * bytes);
  return 0;
}
