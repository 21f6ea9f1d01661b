// Access-pattern probe (tools only, not product code): two rounds of the
// nibble path's loads (gprobe2 mode 0: own lag + age words in, 4 sender lag
// words of the same tile slice, lag + age out) run tile group by tile
// group: round r over tiles [g, g + G) (A -> B), then round r + 1 over the
// same tiles (B -> A), so that round r + 1 reads what round r just wrote
// while it may still sit in the Infinity Cache. G = 256: two whole passes.
//   hipcc -O3 --offload-arch=gfx950 tools/r05/gprobe3.hip -o tools/bin/gprobe3
// G = 0: two whole passes, the second in reverse tile order (it starts on
// the tiles the first pass wrote last).
//   tools/bin/gprobe3 <G tiles per group>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LDS __attribute__((address_space(3)))
#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int N = 65536, TW = 256, RB = 256, NT = N / TW;
constexpr int64_t SLICE = (int64_t)N * (TW / 2);
constexpr int64_t PLANE = SLICE * NT;

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t u = ((uint64_t)(uint32_t)uni((int)(a >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)a);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, (int)SLICE, 0x00020000);
}
__device__ __forceinline__ uint32_t pkmin(uint32_t p, uint32_t r) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, p), __builtin_bit_cast(u16x2, r)));
}
__device__ __forceinline__ uint32_t rule(uint32_t q, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) {
  uint32_t L = 0;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const uint32_t M = 0x000F000Fu << (4 * f);
    L |= pkmin(pkmin(pkmin(q & M, s0 & M), pkmin(s1 & M, s2 & M)), s3 & M);
  }
  return L;
}


__global__ __launch_bounds__(256) void k_probe(const char* __restrict__ lag_in, const char* __restrict__ age_in,
                                               char* __restrict__ lag_out, char* __restrict__ age_out, int round,
                                               int t0, int rev) {
  const int bid = blockIdx.x;
  constexpr int nrb = N / RB;
  const int x = bid & 7, j = bid >> 3;
  const int tf = t0 + x + 8 * (j / nrb), rb = j % nrb;
  const int tile = rev ? NT - 1 - tf : tf;
  const int tid = threadIdx.x, lane = tid & 63, wave = uni(tid >> 6);
  const auto lo = rsrc(lag_in + (int64_t)tile * SLICE);
  const auto ao = rsrc(age_in + (int64_t)tile * SLICE);
  const auto ln = rsrc(lag_out + (int64_t)tile * SLICE);
  const auto an = rsrc(age_out + (int64_t)tile * SLICE);
  uint32_t acc = 0;
  const int sub = lane >> 4, lc = lane & 15;
  const uint32_t lbp = (uint32_t)lc * 8;
#pragma unroll 1
  for (int it = 0; it < RB / 16; it += 2) {
    u32x2 q[2], a[2], s[2][4];
    uint32_t off[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = rb * RB + (it + u) * 16 + wave * 4 + sub;
      off[u] = (uint32_t)row * 128 + lbp;
      a[u] = __builtin_amdgcn_raw_buffer_load_b64(ao, (int)off[u], 0, 2);
      q[u] = __builtin_amdgcn_raw_buffer_load_b64(lo, (int)off[u], 0, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t sr = hash3((uint32_t)row, (uint32_t)k, (uint32_t)round) & (N - 1);
        s[u][k] = __builtin_amdgcn_raw_buffer_load_b64(lo, (int)(sr * 128 + lbp), 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      u32x2 m, g;
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        m[w] = rule(q[u][w], s[u][0][w], s[u][1][w], s[u][2][w], s[u][3][w]);
        g[w] = a[u][w] + 0x11111111u;
        acc += m[w];
      }
      __builtin_amdgcn_raw_buffer_store_b64(m, ln, (int)off[u], 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(g, an, (int)off[u], 0, 2);
    }
  }
  if (acc == 0x9E3779B1u) lag_out[0] = 1;
}

int main(int argc, char** argv) {
  const int G0 = argc > 1 ? atoi(argv[1]) : 256;
  const int G = G0 == 0 ? NT : G0;
  if (G < 8 || G > NT || NT % G || G % 8) {
    fprintf(stderr, "G must be a multiple of 8 dividing %d\n", NT);
    return 2;
  }
  const int reps = 8;
  char *lag[2], *age[2];
  for (int b = 0; b < 2; ++b) {
    CK(hipMalloc(&lag[b], PLANE));
    CK(hipMalloc(&age[b], PLANE));
    CK(hipMemset(lag[b], 0x35, PLANE));
    CK(hipMemset(age[b], 0x22, PLANE));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  const dim3 grid(G * (N / RB));
  for (int l = 0; l < reps + 1; ++l) {
    CK(hipEventRecord(e0));
    for (int t0 = 0; t0 < NT; t0 += G)
      for (int h = 0; h < 2; ++h)
        hipLaunchKernelGGL(k_probe, grid, dim3(256), 0, 0, lag[h], age[h], lag[h ^ 1], age[h ^ 1], 2 * l + h, t0,
                           G0 == 0 ? h : 0);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t = 0.f;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (l) ms.push_back(t / 2);  // per round
  }
  std::sort(ms.begin(), ms.end());
  printf("{\"G\": %d, \"reverse_odd\": %d, \"launches_per_round\": %d, \"ms_per_round_median\": %.4f, \"ms_per_round_min\": %.4f}\n", G, G0 == 0, NT / G,
         ms[ms.size() / 2], ms[0]);
  return 0;
}
