// gr_scan.h — device-wide exclusive scan (hand-written, no library), shared by
// the engine's boundary passes (gr_io.h, gr_engine.hip) and the wire codec
// (gr_wire.hip). Three launches over tiles of kScanTile values: scan_tiles
// (each tile's sum), scan_spine (one block scans the tile sums in place),
// scan_apply (each tile's own scan plus its offset). Blocks of kScanBlock threads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gr {
namespace scan {

constexpr uint32_t kScanBlock = 256, kScanItems = 8, kScanTile = kScanBlock * kScanItems;
// Exclusive scan of one value per thread over the 256-thread block (wave
// shuffles, then the four wave totals through LDS); *total = the block's sum.
template <class T>
__device__ inline T block_excl_scan(T v, T* lds4, T* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const T y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) lds4[w] = x;
  __syncthreads();
  T off = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanBlock / 64; ++k) {
    off += k < w ? lds4[k] : (T)0;
    tot += lds4[k];
  }
  __syncthreads();  // lds4 may be reused by the caller's next call
  *total = tot;
  return off + x - v;
}
template <class T>
__global__ void scan_tiles(const T* in, uint32_t n, T* tile_sum) {
  __shared__ T lds4[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  T s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) s += base + k < n ? in[base + k] : (T)0;
  T tot;
  (void)block_excl_scan(s, lds4, &tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}
// One block: the exclusive scan of the ntiles tile sums, in place.
template <class T>
__global__ void scan_spine(T* tile_sum, uint32_t ntiles) {
  __shared__ T lds4[kScanBlock / 64];
  T carry = 0;
  for (uint32_t b = 0; b < ntiles; b += kScanBlock) {
    const uint32_t t = b + threadIdx.x;
    const T v = t < ntiles ? tile_sum[t] : (T)0;
    T tot;
    const T e = block_excl_scan(v, lds4, &tot);
    if (t < ntiles) tile_sum[t] = carry + e;
    carry += tot;
  }
}
template <class T>
__global__ void scan_apply(const T* in, T* out, uint32_t n, const T* tile_off) {
  __shared__ T lds4[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  T v[kScanItems];
  T s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    v[k] = base + k < n ? in[base + k] : (T)0;
    s += v[k];
  }
  T tot;
  T run = tile_off[blockIdx.x] + block_excl_scan(s, lds4, &tot);
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
}

// Tiles of n values (the grid of scan_tiles and scan_apply, the tile sums' count).
inline uint32_t scan_tiles_of(uint64_t n) { return (uint32_t)((n + kScanTile - 1) / kScanTile); }
// The three launches on `s`; tile_sum has scan_tiles_of(n) elements of scratch.
template <class T>
inline hipError_t exclusive_scan(const T* in, T* out, uint32_t n, T* tile_sum, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t tiles = scan_tiles_of(n);
  hipLaunchKernelGGL(scan_tiles<T>, dim3(tiles), dim3(kScanBlock), 0, s, in, n, tile_sum);
  hipLaunchKernelGGL(scan_spine<T>, dim3(1), dim3(kScanBlock), 0, s, tile_sum, tiles);
  hipLaunchKernelGGL(scan_apply<T>, dim3(tiles), dim3(kScanBlock), 0, s, in, out, n, (const T*)tile_sum);
  return hipGetLastError();
}

}  // namespace scan
}  // namespace gr
