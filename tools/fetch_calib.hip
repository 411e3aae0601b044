// FETCH_SIZE calibration for the access widths the validate kernel issues
// (MI355X_MICROARCH.md §HBM: "calibrate on a known byte count in your own
// access pattern").  Four kernels, each launched once after a warm-up launch,
// on known byte counts:
//   stream16      1 GiB read as 16 B per lane, coalesced (the guide's case:
//                 FETCH_SIZE should read half of it)
//   gather16_cold 2^24 random 16-B gathers over a 4 GiB buffer (beyond the
//                 256 MB Infinity Cache: nearly every gather its own line)
//   gather16_tab  2^24 random 16-B gathers over an 8 MiB table (the x-pair
//                 terrain's size at 1024^2), Infinity-Cache resident
//   rows144       2^18 rows of 144 B read by one lane each, consecutive rows
//                 in consecutive lanes (the attempt-row refill pattern)
// Run under `rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib` and divide each
// kernel's FETCH_SIZE (KiB) by the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

__global__ void stream16(const float4 *__restrict__ a, size_t n4, float *out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[threadIdx.x] = s;
}

// every thread issues PER gathers, all independent (indices from a hash)
template <int PER>
__global__ void gather16(const float4 *__restrict__ a, uint64_t n4, uint64_t salt, float *out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    float4 v = a[mix(t * PER + k + salt) % n4];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[threadIdx.x] = s;
}

__global__ void rows144(const double *__restrict__ rows, int n, float *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double *r = rows + (size_t)i * 18;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 18; ++k) s += r[k];
  if (s == 1234.5) out[threadIdx.x] = (float)s;
}

int main() {
  const size_t big = (size_t)4 << 30, tab = (size_t)8 << 20, stream_bytes = (size_t)1 << 30;
  const uint64_t gathers = 1ull << 24;
  const int nrows = 1 << 18;
  float4 *a = nullptr, *t = nullptr;
  double *rows = nullptr;
  float *out = nullptr;
  CHK(hipMalloc(&a, big));
  CHK(hipMalloc(&t, tab));
  CHK(hipMalloc(&rows, (size_t)nrows * 144));
  CHK(hipMalloc(&out, 4096));
  CHK(hipMemset(a, 0, big));
  CHK(hipMemset(t, 0, tab));
  CHK(hipMemset(rows, 0, (size_t)nrows * 144));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto timed = [&](const char *name, double bytes, auto launch) -> int {
    launch(0);                                   // warm-up (tables become cache resident)
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    launch(1);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"kernel\": \"%s\", \"bytes_requested\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n",
                name, bytes, ms, bytes / (ms * 1e6));
    return 0;
  };
  const int grid = 256 * 8;
  if (timed("stream16", (double)stream_bytes, [&](int) {
        stream16<<<grid, 256>>>(a, stream_bytes / 16, out); })) return 1;
  // distinct salts per launch so the measured launch touches new lines
  if (timed("gather16_cold", 16.0 * gathers, [&](int k) {
        gather16<16><<<gathers / 16 / 256, 256>>>(a, big / 16, 0x9e3779b97f4a7c15ull * (k + 1), out); }))
    return 1;
  if (timed("gather16_tab", 16.0 * gathers, [&](int k) {
        gather16<16><<<gathers / 16 / 256, 256>>>(t, tab / 16, 0x9e3779b97f4a7c15ull * (k + 7), out); }))
    return 1;
  if (timed("rows144", 144.0 * nrows, [&](int) {
        rows144<<<nrows / 256, 256>>>(rows, nrows, out); })) return 1;
  CHK(hipFree(a));
  CHK(hipFree(t));
  CHK(hipFree(rows));
  CHK(hipFree(out));
  return 0;
}
