// Access-pattern probe (tools only, not product code): the nibble path's
// loads (own lag + age words in, 4 sender lag words of the same tile slice,
// lag + age out; N = 65,536, TW = 256) with the sender gathers split over
// lane halves:
//   mode 0: as built: a lane owns 16 cells and loads 8 B of each of its
//           row's 4 senders (4 gathers per row step, each wave instruction
//           touching 4 lines)
//   mode 1: lanes m and m + 8 of a row's 16 share 32 cells: lane m loads
//           16 B of senders 0 and 1, lane m + 8 the same bytes of senders 2
//           and 3 (2 gathers per row step, each touching 8 lines); each
//           takes the per-nibble min of its two, the halves swap by DPP
//           (row_ror 8), and each lane finishes its own 16 cells; own loads
//           and stores as in mode 0
//   hipcc -O3 --offload-arch=gfx950 tools/r05/gprobe4.hip -o tools/bin/gprobe4
//   tools/bin/gprobe4 <mode>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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
// per-nibble min of two words (4 masked fields, one per 16-bit half each)
__device__ __forceinline__ uint32_t nmin2(uint32_t a, uint32_t b) {
  uint32_t L = 0;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const uint32_t M = 0x000F000Fu << (4 * f);
    L |= pkmin(a & M, b & M);
  }
  return L;
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
__device__ __forceinline__ uint32_t rule3(uint32_t q, uint32_t a, uint32_t b) {
  uint32_t L = 0;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const uint32_t M = 0x000F000Fu << (4 * f);
    L |= pkmin(pkmin(q & M, a & M), b & M);
  }
  return L;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const char* __restrict__ lag_in, const char* __restrict__ age_in,
                                               char* __restrict__ lag_out, char* __restrict__ age_out, int round) {
  const int bid = blockIdx.x;
  constexpr int nrb = N / RB;
  const int x = bid & 7, j = bid >> 3;
  const int tile = x + 8 * (j / nrb), rb = j % nrb;
  const int tid = threadIdx.x, lane = tid & 63, wave = uni(tid >> 6);
  const auto lo = rsrc(lag_in + (int64_t)tile * SLICE);
  const auto ao = rsrc(age_in + (int64_t)tile * SLICE);
  const auto ln = rsrc(lag_out + (int64_t)tile * SLICE);
  const auto an = rsrc(age_out + (int64_t)tile * SLICE);
  uint32_t acc = 0;
  const int sub = lane >> 4, lc = lane & 15;
  // mode 0: the lane's 8 B at lc * 8; mode 1: lane m = lc % 8, half g = lc / 8
  // owns bytes m * 16 + g * 8 (its 16 cells), gathers 16 B at m * 16
  const int m = lc & 7, g = lc >> 3;
  const uint32_t lbp = MODE == 0 ? (uint32_t)lc * 8 : (uint32_t)(m * 16 + g * 8);
  const uint32_t gbp = (uint32_t)m * 16;
#pragma unroll 1
  for (int it = 0; it < RB / 16; it += 2) {
    u32x2 q[2], a[2], s[2][4];
    u32x4 h[2][2];
    uint32_t off[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = rb * RB + (it + u) * 16 + wave * 4 + sub;
      off[u] = (uint32_t)row * 128 + lbp;
      a[u] = __builtin_amdgcn_raw_buffer_load_b64(ao, (int)off[u], 0, 2);
      q[u] = __builtin_amdgcn_raw_buffer_load_b64(lo, (int)off[u], 0, 0);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t sr = hash3((uint32_t)row, (uint32_t)k, (uint32_t)round) & (N - 1);
          s[u][k] = __builtin_amdgcn_raw_buffer_load_b64(lo, (int)(sr * 128 + lbp), 0, 0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint32_t sr = hash3((uint32_t)row, (uint32_t)(2 * g + t), (uint32_t)round) & (N - 1);
          h[u][t] = __builtin_amdgcn_raw_buffer_load_b128(lo, (int)(sr * 128 + gbp), 0, 0);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      u32x2 mm, ag;
      if constexpr (MODE == 0) {
#pragma unroll
        for (int w = 0; w < 2; ++w) mm[w] = rule(q[u][w], s[u][0][w], s[u][1][w], s[u][2][w], s[u][3][w]);
      } else {
        // the min of my two senders over the 32 cells, then the partner's
        uint32_t pm[4], pp[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          pm[w] = nmin2(h[u][0][w], h[u][1][w]);
          pp[w] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pm[w], 0x128, 0xF, 0xF, false);  // row_ror:8
        }
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          const uint32_t mine = g ? pm[2 + w] : pm[w];
          const uint32_t theirs = g ? pp[2 + w] : pp[w];
          mm[w] = rule3(q[u][w], mine, theirs);
        }
      }
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        ag[w] = a[u][w] + 0x11111111u;
        acc += mm[w];
      }
      __builtin_amdgcn_raw_buffer_store_b64(mm, ln, (int)off[u], 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(ag, an, (int)off[u], 0, 2);
    }
  }
  if (acc == 0x9E3779B1u) lag_out[0] = 1;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int launches = 12;
  char *lag[2], *age[2];
  for (int b = 0; b < 2; ++b) {
    CK(hipMalloc(&lag[b], PLANE));
    CK(hipMalloc(&age[b], PLANE));
    CK(hipMemset(lag[b], 0x35, PLANE));
    CK(hipMemset(age[b], 0x22, PLANE));
  }
  // mode 1 against mode 0 on a small random input: the same outputs
  {
    std::vector<uint8_t> h(PLANE);
    uint32_t st = 12345;
    for (int64_t i = 0; i < PLANE; ++i) {
      st = st * 1664525u + 1013904223u;
      h[i] = (uint8_t)(st >> 24);
    }
    CK(hipMemcpy(lag[0], h.data(), PLANE, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_probe<0>, dim3(NT * (N / RB)), dim3(256), 0, 0, lag[0], age[0], lag[1], age[1], 7);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> r0(PLANE), r1(PLANE);
    CK(hipMemcpy(r0.data(), lag[1], PLANE, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(k_probe<1>, dim3(NT * (N / RB)), dim3(256), 0, 0, lag[0], age[0], lag[1], age[1], 7);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r1.data(), lag[1], PLANE, hipMemcpyDeviceToHost));
    if (r0 != r1) {
      fprintf(stderr, "mode 1 differs from mode 0\n");
      return 3;
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  const dim3 grid(NT * (N / RB));
  for (int l = 0; l < launches + 1; ++l) {
    const int c = l & 1;
    CK(hipEventRecord(e0));
    if (mode == 0)
      hipLaunchKernelGGL(k_probe<0>, grid, dim3(256), 0, 0, lag[c], age[c], lag[c ^ 1], age[c ^ 1], l);
    else
      hipLaunchKernelGGL(k_probe<1>, grid, dim3(256), 0, 0, lag[c], age[c], lag[c ^ 1], age[c ^ 1], l);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t = 0.f;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (l) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  printf("{\"mode\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f}\n", mode, ms[ms.size() / 2], ms[0]);
  return 0;
}
