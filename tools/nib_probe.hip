// Timing + PMC-calibration probe (not product code) for the nibble path's
// access pattern at N=65,536: 256 tiles of TW = 256 members, per tile a lag
// plane slice and an age plane slice of N rows x 128 B (4 bits per cell), in
// and out (double-buffered, 8 GiB). Modes:
//   0 stream  : own lag + age words in (4 B per lane), out; no gathers
//   1 gather  : mode 0 + k = 4 random sender lag words per row (the same tile
//               slice), trivial nibble min merge
//   2 rd4     : plain streaming read of the 4 GiB in-planes, 4 B per lane
//   3 rd16    : the same, 16 B per lane (the guide's calibrated width)
//   4 wr4     : plain streaming write of the 4 GiB out-planes, 4 B per lane
// Prints ms per launch (HIP events, median of 10) and the algorithmic bytes,
// so rocprofv3 --pmc runs of one mode calibrate FETCH_SIZE / TCC_EA0_RDREQ
// against a known byte count at this access width (MI355X_MICROARCH.md:
// "other access widths are uncalibrated").
//   hipcc -O3 --offload-arch=gfx950 tools/nib_probe.hip -o tools/bin/nib_probe
//   tools/bin/nib_probe <mode> [launches]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int N = 65536, TW = 256, RB = 256, NT = N / TW;
constexpr int64_t SLICE = (int64_t)N * (TW / 2);  // bytes per tile slice of one plane
constexpr int64_t PLANE = SLICE * NT;             // 2 GiB

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}
// buffer resource of one tile slice (gfx9 dword3; loads past num_records return 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char* p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)SLICE, 0x00020000);
}
#define LD(r, off, aux) __builtin_amdgcn_raw_buffer_load_b32((r), (int)(off), 0, (aux))
#define ST(v, r, off, aux) __builtin_amdgcn_raw_buffer_store_b32((v), (r), (int)(off), 0, (aux))

template <bool GATHER>
__global__ __launch_bounds__(256) void k_nib(const char* __restrict__ lag_in, const char* __restrict__ age_in,
                                             char* __restrict__ lag_out, char* __restrict__ age_out, int round) {
  const int bid = blockIdx.x;
  constexpr int nrb = N / RB;
  const int x = bid & 7, j = bid >> 3;
  const int tile = x + 8 * (j / nrb), rb = j % nrb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = lane >> 5, lc = lane & 31;
  const auto lo = rsrc(lag_in + (int64_t)tile * SLICE);
  const auto ao = rsrc(age_in + (int64_t)tile * SLICE);
  const auto ln = rsrc(lag_out + (int64_t)tile * SLICE);
  const auto an = rsrc(age_out + (int64_t)tile * SLICE);
  uint32_t acc = 0;
#pragma unroll 1
  for (int it = 0; it < RB / 8; it += 2) {
    uint32_t q[2], a[2], s[2][4];
    uint32_t off[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = rb * RB + (it + u) * 8 + wave * 2 + sub;
      off[u] = (uint32_t)row * 128u + (uint32_t)lc * 4u;
      a[u] = LD(ao, off[u], 2);
      q[u] = LD(lo, off[u], 0);
      if constexpr (GATHER) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t sr = hash3((uint32_t)row, (uint32_t)k, (uint32_t)round) & (N - 1);
          s[u][k] = LD(lo, sr * 128u + (uint32_t)lc * 4u, 0);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t m = q[u];
      if constexpr (GATHER) {
        uint32_t L = 0;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const uint32_t M = 0x000F000Fu << (4 * f);
          const auto mn = [](uint32_t p, uint32_t r) {
            return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, p),
                                                                          __builtin_bit_cast(u16x2, r)));
          };
          L |= mn(mn(s[u][0] & M, s[u][1] & M), mn(s[u][2] & M, s[u][3] & M));
        }
        m = L ^ q[u];
      }
      ST(m, ln, off[u], 2);
      ST(a[u] + 0x11111111u, an, off[u], 2);
      acc += m;
    }
  }
  if (acc == 0x9E3779B1u) lag_out[0] = 1;
}

template <int W>
__global__ __launch_bounds__(256) void k_rd(const uint32_t* __restrict__ p, int64_t nwords, uint32_t* out) {
  typedef uint32_t vw __attribute__((ext_vector_type(W)));
  uint32_t acc = 0;
  const int64_t nv = nwords / W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const vw v = __builtin_nontemporal_load(reinterpret_cast<const vw*>(p) + i);
#pragma unroll
    for (int w = 0; w < W; ++w) acc ^= v[w];
  }
  if (acc == 0x9E3779B1u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_wr4(uint32_t* __restrict__ p, int64_t nwords, uint32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(v + (uint32_t)i, p + i);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 1;
  const int launches = argc > 2 ? atoi(argv[2]) : 10;
  char *lag[2], *age[2];
  for (int b = 0; b < 2; ++b) {
    CK(hipMalloc(&lag[b], PLANE));
    CK(hipMalloc(&age[b], PLANE));
    CK(hipMemset(lag[b], 0x35, PLANE));
    CK(hipMemset(age[b], 0x22, PLANE));
  }
  uint32_t* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int64_t nwords = 2 * PLANE / 4;  // mode 2-4: both planes of a buffer (they are separate allocations)
  double bytes = 0;
  std::vector<float> ms;
  for (int l = 0; l < launches + 1; ++l) {
    const int c = l & 1;
    CK(hipEventRecord(e0));
    switch (mode) {
      case 0:
      case 1: {
        const dim3 grid(NT * (N / RB));
        if (mode == 0)
          hipLaunchKernelGGL(k_nib<false>, grid, dim3(256), 0, 0, lag[c], age[c], lag[c ^ 1], age[c ^ 1], l);
        else
          hipLaunchKernelGGL(k_nib<true>, grid, dim3(256), 0, 0, lag[c], age[c], lag[c ^ 1], age[c ^ 1], l);
        bytes = 4.0 * (double)PLANE;  // lag + age in and out (gathers are extra)
        break;
      }
      case 2:
        hipLaunchKernelGGL(k_rd<1>, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(lag[c]), nwords / 2, out);
        hipLaunchKernelGGL(k_rd<1>, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(age[c]), nwords / 2, out);
        bytes = 2.0 * (double)PLANE;
        break;
      case 3:
        hipLaunchKernelGGL(k_rd<4>, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(lag[c]), nwords / 2, out);
        hipLaunchKernelGGL(k_rd<4>, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(age[c]), nwords / 2, out);
        bytes = 2.0 * (double)PLANE;
        break;
      default:
        hipLaunchKernelGGL(k_wr4, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(lag[c]), nwords / 2, 7u);
        hipLaunchKernelGGL(k_wr4, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(age[c]), nwords / 2, 9u);
        bytes = 2.0 * (double)PLANE;
        break;
    }
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t = 0.f;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (l) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double med = ms[ms.size() / 2];
  printf("{\"mode\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"bytes\": %.0f, \"gbs\": %.1f}\n", mode, med, ms[0],
         bytes, bytes / med / 1e6);
  return 0;
}
