// FETCH_SIZE calibration for the table lookup's access patterns (not part of
// the library).  MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for wide coalesced streaming
// reads (it reports 1/2 of the bytes); the lookup reads random 64-byte pair records (four 16-byte
// loads per lane, lk_pair in csrc/airice_lookup.hpp) and random 32-byte pieces of its 256-byte row
// records (lk_row_rec).  Each probe below reads a KNOWN number of bytes in one of those patterns;
// rocprofv3 --pmc FETCH_SIZE of each dispatch against that count gives the pattern's factor
// (tools/fetch_calib.py).  Every random probe visits each record of its draw exactly once (a
// bijective hash of the lane index), so no record is read twice in a launch.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
//   tools/fetch_calib [json_out]        (prints one JSON object: probes, bytes, times)
//
// Probes (each launched kReps times after one warm-up launch; a dispatch reads its bytes once):
//   stream16     : 16 B per lane, coalesced, over a 2 GiB buffer (the guide's calibrated case)
//   wstream16    : 16 B per lane stored, coalesced, 2 GiB (the streaming write rate; timing only)
//   rand64_big   : one random 64-byte record per lane (4 x float4), 2^24 draws from 2^25 records
//                  of a 2 GiB table -- larger than the 256 MiB Infinity Cache
//   rand32_big   : one random 32-byte piece (2 x float4) of a random 256-byte record, 2 GiB table
//   rand64_small : as rand64_big on a 96 MiB table (1.5M records, the size of the cfg2 lookup's
//                  packed table), L3-resident after the warm-up: what FETCH_SIZE counts for
//                  Infinity-Cache hits
// Each lane folds what it read into one float; one float per wave is stored (negligible writes).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr int kBlock = 256;
constexpr int kReps = 5;

// a bijection of [0, 2^bits): odd multiply, xor-shift, odd multiply (each invertible mod 2^bits)
__device__ __forceinline__ uint32_t scatter(uint32_t i, int bits) {
  const uint32_t m = (bits == 32) ? 0xffffffffu : ((1u << bits) - 1u);
  uint32_t x = (i * 0x9E3779B1u) & m;
  x ^= x >> (bits / 2);
  x = (x * 0x85EBCA77u) & m;
  x ^= x >> (bits / 3 + 1);
  return x & m;
}

__device__ __forceinline__ void wave_out(float v, float* out) {
  // one float per wave: the lanes' sum through shuffles
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) out[(blockIdx.x * kBlock + threadIdx.x) >> 6] = v;
}

__global__ __launch_bounds__(kBlock) void stream16(const float4* __restrict__ a, long long n,
                                                    float* out) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  float v = 0.f;
  if (i < n) {
    const float4 x = a[i];
    v = x.x + x.y + x.z + x.w;
  }
  wave_out(v, out);
}

// 16 B per lane stored, coalesced: the streaming write rate (the lookup's result columns)
__global__ __launch_bounds__(kBlock) void wstream16(float4* __restrict__ a, long long n) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) a[i] = float4{(float)i, 1.f, 2.f, 3.f};
}

// lane i reads record scatter(i) of 64 B: four 16-byte loads at p[0..3], as lk_pair does
__global__ __launch_bounds__(kBlock) void rand64(const float4* __restrict__ t, int bits,
                                                  long long draws, float* out) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  float v = 0.f;
  if (i < draws) {
    const float4* p = t + 4ll * scatter((uint32_t)i, bits);
    const float4 a = p[0], b = p[1], c = p[2], d = p[3];
    v = a.x + b.y + c.z + d.w;
  }
  wave_out(v, out);
}

// lane i reads the first 32 B (two 16-byte loads) of 256-byte record scatter(i), as lk_row_rec
__global__ __launch_bounds__(kBlock) void rand32(const float4* __restrict__ t, int bits,
                                                  long long draws, float* out) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  float v = 0.f;
  if (i < draws) {
    const float4* p = t + 16ll * scatter((uint32_t)i, bits);
    const float4 a = p[0], b = p[1];
    v = a.x + b.w;
  }
  wave_out(v, out);
}

// rand64 over a table of `records` records that is not a power of two: draws of the bijection on
// 2^bits >= records that fall outside are skipped (each record still read at most once)
__global__ __launch_bounds__(kBlock) void rand64_n(const float4* __restrict__ t, int bits,
                                                    long long records, float* out,
                                                    unsigned long long* hits) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  float v = 0.f;
  const uint32_t r = scatter((uint32_t)i, bits);
  const bool take = i < (1ll << bits) && r < (uint64_t)records;
  if (take) {
    const float4* p = t + 4ll * r;
    const float4 a = p[0], b = p[1], c = p[2], d = p[3];
    v = a.x + b.y + c.z + d.w;
  }
  if (hits != nullptr) {  // the check launch only: one atomic per wave would serialise the timing
    const unsigned long long m = __ballot(take);
    if ((threadIdx.x & 63) == 0) atomicAdd(hits, (unsigned long long)__popcll(m));
  }
  wave_out(v, out);
}

struct Probe {
  std::string name;
  double bytes;  // bytes the probe's loads request per launch
  float ms;      // mean per launch
  long long lanes;
};

int main(int argc, char** argv) {
  const size_t big = 2ull << 30;  // 2 GiB
  float4* buf = nullptr;
  float* out = nullptr;
  unsigned long long* hits = nullptr;
  CHECK(hipMalloc(&buf, big));
  CHECK(hipMemset(buf, 0, big));  // defined values (the sums are never checked)
  CHECK(hipMalloc(&out, sizeof(float) * ((1ll << 27) / 64 + 64)));  // one float per wave
  CHECK(hipMalloc(&hits, sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<Probe> probes;

  auto timed = [&](const char* name, double bytes, long long lanes, auto launch) -> int {
    launch();  // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < kReps; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    probes.push_back(Probe{name, bytes, ms / kReps, lanes});
    return 0;
  };

  {  // stream16: 2^27 lanes x 16 B = 2 GiB
    const long long n = (long long)(big / 16);
    const unsigned g = (unsigned)((n + kBlock - 1) / kBlock);
    if (timed("stream16", 16.0 * n, n, [&] {
          hipLaunchKernelGGL(stream16, dim3(g), dim3(kBlock), 0, 0, buf, n, out);
        }))
      return 1;
  }
  {  // wstream16: 2^27 lanes x 16 B = 2 GiB written
    const long long n = (long long)(big / 16);
    const unsigned g = (unsigned)((n + kBlock - 1) / kBlock);
    if (timed("wstream16", 16.0 * n, n, [&] {
          hipLaunchKernelGGL(wstream16, dim3(g), dim3(kBlock), 0, 0, buf, n);
        }))
      return 1;
  }
  {  // rand64_big: 2^24 draws of 64 B from 2^25 records (2 GiB)
    const int bits = 25;
    const long long draws = 1ll << 24;
    const unsigned g = (unsigned)(draws / kBlock);
    if (timed("rand64_big", 64.0 * draws, draws, [&] {
          hipLaunchKernelGGL(rand64, dim3(g), dim3(kBlock), 0, 0, buf, bits, draws, out);
        }))
      return 1;
  }
  {  // rand32_big: 2^23 draws of 32 B from 2^23 records of 256 B (2 GiB)
    const int bits = 23;
    const long long draws = 1ll << 23;
    const unsigned g = (unsigned)(draws / kBlock);
    if (timed("rand32_big", 32.0 * draws, draws, [&] {
          hipLaunchKernelGGL(rand32, dim3(g), dim3(kBlock), 0, 0, buf, bits, draws, out);
        }))
      return 1;
  }
  {  // rand64_small: every record of a 96 MiB table once per launch (1,572,864 records)
    const long long records = (96ll << 20) / 64;
    const int bits = 21;  // 2^21 >= records
    const long long lanes = 1ll << bits;
    const unsigned g = (unsigned)(lanes / kBlock);
    CHECK(hipMemset(hits, 0, sizeof(unsigned long long)));
    hipLaunchKernelGGL(rand64_n, dim3(g), dim3(kBlock), 0, 0, buf, bits, records, out, hits);
    unsigned long long h = 0;
    CHECK(hipMemcpy(&h, hits, sizeof(h), hipMemcpyDeviceToHost));
    if ((long long)h != records) {
      std::fprintf(stderr, "rand64_small: %llu records taken, want %lld\n", h, records);
      return 1;
    }
    if (timed("rand64_small", 64.0 * records, lanes, [&] {
          hipLaunchKernelGGL(rand64_n, dim3(g), dim3(kBlock), 0, 0, buf, bits, records, out,
                             (unsigned long long*)nullptr);
        }))
      return 1;
  }

  std::string js = "{\"reps\": " + std::to_string(kReps) + ", \"warmup\": 1, \"probes\": [";
  for (size_t i = 0; i < probes.size(); ++i) {
    char line[512];
    std::snprintf(line, sizeof line,
                  "%s{\"name\": \"%s\", \"bytes_per_launch\": %.0f, \"lanes\": %lld, "
                  "\"ms\": %.5f, \"GBps\": %.1f}",
                  i ? ", " : "", probes[i].name.c_str(), probes[i].bytes, probes[i].lanes,
                  probes[i].ms, probes[i].bytes / (probes[i].ms * 1e-3) / 1e9);
    js += line;
  }
  js += "]}";
  std::printf("%s\n", js.c_str());
  if (argc > 1) {
    if (FILE* f = std::fopen(argv[1], "w")) {
      std::fprintf(f, "%s\n", js.c_str());
      std::fclose(f);
    }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  CHECK(hipFree(hits));
  return 0;
}
