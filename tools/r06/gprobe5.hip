// Access-pattern probe (tools only, not product code): the nibble path's
// own streams as one 16-B load and one 16-B store per lane and row step
// instead of two 8-B loads and two 8-B stores (N = 65,536, TW = 256, 4
// sender gathers of 8 B per lane as built):
//   mode 0: as built: lag and age planes in two buffers; a lane owns 16 cells
//           and loads 8 B of each (two own loads, two stores per row step)
//   mode 2: each tile's lag slice followed by its age slice in ONE buffer
//           (one buffer resource covers both); lanes m and m + 8 of a row
//           share 32 cells: lane m loads their 16 B of lag, lane m + 8 their
//           16 B of age, one DPP swap (row_ror 8) gives each lane the lag and
//           age of its own 16 cells; stores the same way in reverse
//   hipcc -O3 --offload-arch=gfx950 tools/r06/gprobe5.hip -o tools/bin/gprobe5
//   tools/bin/gprobe5 <mode>
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
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t u = ((uint64_t)(uint32_t)uni((int)(a >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)a);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, (int)bytes, 0x00020000);
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
__device__ __forceinline__ uint32_t swap8(uint32_t x) {  // lane m <-> m + 8 of each 16-lane row
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);
}

// mode 0: lag_in / age_in / lag_out / age_out are separate planes; mode 2:
// lag_in (= in) holds per tile [lag slice | age slice], lag_out likewise
template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const char* __restrict__ lag_in, const char* __restrict__ age_in,
                                               char* __restrict__ lag_out, char* __restrict__ age_out, int round) {
  const int bid = blockIdx.x;
  constexpr int nrb = N / RB;
  const int x = bid & 7, j = bid >> 3;
  const int tile = x + 8 * (j / nrb), rb = j % nrb;
  const int tid = threadIdx.x, lane = tid & 63, wave = uni(tid >> 6);
  const int64_t tstride = MODE == 2 ? 2 * SLICE : SLICE;
  const auto lo = rsrc(lag_in + (int64_t)tile * tstride, tstride);
  const auto ao = rsrc(age_in + (int64_t)tile * SLICE, SLICE);
  const auto ln = rsrc(lag_out + (int64_t)tile * tstride, tstride);
  const auto an = rsrc(age_out + (int64_t)tile * SLICE, SLICE);
  uint32_t acc = 0;
  const int sub = lane >> 4, lc = lane & 15;
  const int m = lc & 7, g = lc >> 3;
  // the lane's 16 cells: mode 0 bytes lc * 8; mode 2 bytes m * 16 + g * 8
  const uint32_t lbp = MODE == 0 ? (uint32_t)lc * 8 : (uint32_t)(m * 16 + g * 8);
  // mode 2: the 16 B this lane moves: lag (g = 0) or age (g = 1) of bytes m * 16
  const uint32_t pbp = (uint32_t)(g ? SLICE : 0) + (uint32_t)m * 16;
#pragma unroll 1
  for (int it = 0; it < RB / 16; it += 2) {
    u32x2 q[2], a[2], s[2][4];
    u32x4 x4[2];
    uint32_t row_b[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = rb * RB + (it + u) * 16 + wave * 4 + sub;
      row_b[u] = (uint32_t)row * 128;
      if constexpr (MODE == 0) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b64(ao, (int)(row_b[u] + lbp), 0, 2);
        q[u] = __builtin_amdgcn_raw_buffer_load_b64(lo, (int)(row_b[u] + lbp), 0, 0);
      } else {
        x4[u] = __builtin_amdgcn_raw_buffer_load_b128(lo, (int)(row_b[u] + pbp), 0, 0);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t sr = hash3((uint32_t)row, (uint32_t)k, (uint32_t)round) & (N - 1);
        s[u][k] = __builtin_amdgcn_raw_buffer_load_b64(lo, (int)(sr * 128 + lbp), 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if constexpr (MODE == 2) {
        // g = 0 holds lag [c0 | c1], g = 1 age [c0 | c1] of the pair's cells;
        // g = 0 computes c0, g = 1 computes c1
        const uint32_t s0 = g ? x4[u][0] : x4[u][2], s1 = g ? x4[u][1] : x4[u][3];
        const uint32_t r0 = swap8(s0), r1 = swap8(s1);
        q[u][0] = g ? r0 : x4[u][0];
        q[u][1] = g ? r1 : x4[u][1];
        a[u][0] = g ? x4[u][2] : r0;
        a[u][1] = g ? x4[u][3] : r1;
      }
      u32x2 mm, ag;
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        mm[w] = rule(q[u][w], s[u][0][w], s[u][1][w], s[u][2][w], s[u][3][w]);
        ag[w] = a[u][w] + 0x11111111u;
        acc += mm[w];
      }
      if constexpr (MODE == 0) {
        __builtin_amdgcn_raw_buffer_store_b64(mm, ln, (int)(row_b[u] + lbp), 0, 18);
        __builtin_amdgcn_raw_buffer_store_b64(ag, an, (int)(row_b[u] + lbp), 0, 18);
      } else {
        // g = 0 stores lag [c0 | c1] (its mm, the partner's), g = 1 age [c0 | c1]
        const uint32_t t0 = g ? mm[0] : ag[0], t1 = g ? mm[1] : ag[1];
        const uint32_t p0 = swap8(t0), p1 = swap8(t1);
        u32x4 o;
        o[0] = g ? p0 : mm[0];
        o[1] = g ? p1 : mm[1];
        o[2] = g ? ag[0] : p0;
        o[3] = g ? ag[1] : p1;
        __builtin_amdgcn_raw_buffer_store_b128(o, ln, (int)(row_b[u] + pbp), 0, 18);
      }
    }
  }
  if (acc == 0x9E3779B1u) lag_out[0] = 1;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int launches = 12;
  char *buf[2], *age[2];
  for (int b = 0; b < 2; ++b) {
    CK(hipMalloc(&buf[b], 2 * PLANE));  // mode 2: both planes, tile-interleaved; mode 0: the lag plane
    CK(hipMalloc(&age[b], PLANE));
    CK(hipMemset(buf[b], 0x35, 2 * PLANE));
    CK(hipMemset(age[b], 0x22, PLANE));
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
      hipLaunchKernelGGL(k_probe<0>, grid, dim3(256), 0, 0, buf[c], age[c], buf[c ^ 1], age[c ^ 1], l);
    else
      hipLaunchKernelGGL(k_probe<2>, grid, dim3(256), 0, 0, buf[c], age[c], buf[c ^ 1], age[c ^ 1], l);
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
