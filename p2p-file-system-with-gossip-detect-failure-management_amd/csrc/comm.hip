// Collective transports of the column-sharded engine (comm.h).
//
// RCCL is opened with dlopen so that libgossiphip loads (and its single-GPU
// path runs) on hosts without RCCL; only a sharded engine created with
// GH_COMM_RCCL needs it.
#include "comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <type_traits>
#include <vector>

size_t gh_dtype_size(GhDType dt) { return dt == GH_DT_U8 ? 1 : dt == GH_DT_I32 ? 4 : 8; }

namespace {

int copy_if_needed(const void* send, void* recv, size_t bytes, hipStream_t s) {
  if (send == recv || bytes == 0) return 0;
  return hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : -1;
}

struct SingleComm final : GhComm {
  int allreduce(const void* send, void* recv, size_t count, GhDType dt, GhROp, hipStream_t s) override {
    return copy_if_needed(send, recv, count * gh_dtype_size(dt), s);
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return copy_if_needed(send, recv, bytes, s);
  }
  int alltoallv(const void* send, const size_t* sendbytes, void* recv, const size_t*, hipStream_t s,
                const size_t* recvdispl) override {
    return copy_if_needed(send, static_cast<char*>(recv) + (recvdispl ? recvdispl[0] : 0), sendbytes[0], s);
  }
};

// ---- RCCL ----------------------------------------------------------------
struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_to_allv)(const void*, const size_t[], const size_t[], void*, const size_t[], const size_t[],
                              ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string load_err;
  bool ok = false;
};

const RcclApi& rccl_api() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
      const char* e = dlerror();
      api.load_err = std::string("cannot load RCCL: ") + (e ? e : "unknown");
      return;
    }
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) api.load_err = std::string("RCCL symbol missing: ") + name;
      return fn != nullptr;
    };
    api.ok = sym(api.get_unique_id, "ncclGetUniqueId") && sym(api.comm_init_rank, "ncclCommInitRank") &&
             sym(api.comm_destroy, "ncclCommDestroy") && sym(api.all_reduce, "ncclAllReduce") &&
             sym(api.all_gather, "ncclAllGather") && sym(api.error_string, "ncclGetErrorString") &&
             sym(api.all_to_allv, "ncclAllToAllv");
  });
  return api;
}

ncclDataType_t nccl_type(GhDType dt) {
  return dt == GH_DT_U8 ? ncclUint8 : dt == GH_DT_I32 ? ncclInt32 : ncclUint64;
}

struct RcclComm final : GhComm {
  const RcclApi* api = nullptr;
  ncclComm_t comm = nullptr;
  ~RcclComm() override {
    if (comm) api->comm_destroy(comm);
  }
  int check(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return 0;
    err = std::string(what) + ": " + api->error_string(r);
    return -1;
  }
  int allreduce(const void* send, void* recv, size_t count, GhDType dt, GhROp op, hipStream_t s) override {
    if (count == 0) return 0;
    return check(api->all_reduce(send, recv, count, nccl_type(dt), op == GH_OP_SUM ? ncclSum : ncclMax, comm, s),
                 "ncclAllReduce");
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (bytes == 0) return 0;
    return check(api->all_gather(send, recv, bytes, ncclUint8, comm, s), "ncclAllGather");
  }
  // ncclAllToAllv (rccl.h:815) over byte counts, displacements = prefix sums
  int alltoallv(const void* send, const size_t* sendbytes, void* recv, const size_t* recvbytes,
                hipStream_t s, const size_t* recvdispl) override {
    std::vector<size_t> sd(world), rd(world);
    size_t so = 0, ro = 0;
    for (int r = 0; r < world; ++r) {
      sd[r] = so;
      rd[r] = recvdispl ? recvdispl[r] : ro;
      so += sendbytes[r];
      ro += recvbytes[r];
    }
    if (so + ro == 0) return 0;
    return check(api->all_to_allv(send, sendbytes, sd.data(), recv, recvbytes, rd.data(), ncclUint8, comm, s),
                 "ncclAllToAllv");
  }
};

// ---- LOCAL (threads of one process) --------------------------------------
struct LocalGroup {
  const int world;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<const void*> ptr;
  std::vector<int> dev;
  std::vector<const size_t*> counts;  // alltoallv: each rank's per-destination byte counts
  explicit LocalGroup(int w) : world(w), ptr(w, nullptr), dev(w, 0), counts(w, nullptr) {}
  // All ranks meet. False after a 120 s wait (a rank failed or diverged);
  // the group then stays broken so that no rank hangs on it later.
  bool barrier() {
    std::unique_lock<std::mutex> l(m);
    if (broken) return false;
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(l, std::chrono::seconds(120), [&] { return gen != g || broken; });
    if (!ok || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

std::mutex g_groups_m;
std::map<std::string, std::weak_ptr<LocalGroup>> g_groups;

template <typename T, int OP>
__global__ __launch_bounds__(256) void k_reduce(const T* __restrict__ parts, int world, size_t count,
                                                T* __restrict__ out) {
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < count; x += (size_t)gridDim.x * blockDim.x) {
    T a = parts[x];
    for (int h = 1; h < world; ++h) {
      const T b = parts[(size_t)h * count + x];
      a = OP == GH_OP_SUM ? (T)(a + b) : (b > a ? b : a);
    }
    out[x] = a;
  }
}

// Same-device ranks (G shards of one GPU): one kernel per collective reads
// the peers' buffers directly, instead of one copy launch per peer (a G=8
// row-shard round had issued ~600 copies)
constexpr int kLocalDirect = 16;  // ranks
struct Segs {
  const char* src[kLocalDirect];
  int64_t dst[kLocalDirect];    // byte offset in recv
  int64_t begin[kLocalDirect + 1];  // prefix sums of the segments' bytes
  int n;
};
template <int W>
__global__ __launch_bounds__(256) void k_copy_segs(Segs g, char* __restrict__ recv) {
  const int64_t total = g.begin[g.n];
  const int64_t units = total / W;
  int h = 0;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = u * W;
    while (b >= g.begin[h + 1]) ++h;  // (monotone per thread)
    while (b < g.begin[h]) --h;
    const int64_t o = b - g.begin[h];
    if constexpr (W == 16)
      *reinterpret_cast<uint4*>(recv + g.dst[h] + o) = *reinterpret_cast<const uint4*>(g.src[h] + o);
    else
      recv[g.dst[h] + o] = g.src[h][o];
  }
}
struct Ptrs {
  const void* p[kLocalDirect];
};
template <typename T, int OP>
__global__ __launch_bounds__(256) void k_reduce_ptrs(Ptrs ps, int world, size_t count, T* __restrict__ out) {
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < count; x += (size_t)gridDim.x * blockDim.x) {
    T a = static_cast<const T*>(ps.p[0])[x];
    for (int h = 1; h < world; ++h) {
      const T b = static_cast<const T*>(ps.p[h])[x];
      a = OP == GH_OP_SUM ? (T)(a + b) : (b > a ? b : a);
    }
    out[x] = a;
  }
}

struct LocalComm final : GhComm {
  std::shared_ptr<LocalGroup> g;
  int device = 0;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  ~LocalComm() override {
    if (tmp) (void)hipFree(tmp);
  }
  int fail(const std::string& m) {
    err = m;
    return -1;
  }
  // every rank on this rank's device (then the direct kernels)
  bool direct() const {
    if (world > kLocalDirect) return false;
    for (int h = 0; h < world; ++h)
      if (g->dev[h] != device) return false;
    return true;
  }
  int meet() { return g->barrier() ? 0 : fail("local comm: barrier timeout (a rank failed or diverged)"); }
  int sync(hipStream_t s) { return hipStreamSynchronize(s) == hipSuccess ? 0 : fail("local comm: stream sync failed"); }
  // recv[dst[h] ..] = segment h, in one launch
  int copy_segs(Segs& sg, char* recv, hipStream_t s) {
    const int64_t total = sg.begin[sg.n];
    if (total == 0) return 0;
    bool al = (reinterpret_cast<uintptr_t>(recv) & 15) == 0;
    for (int h = 0; h < sg.n; ++h)
      al = al && (reinterpret_cast<uintptr_t>(sg.src[h]) & 15) == 0 && sg.dst[h] % 16 == 0 &&
           (sg.begin[h + 1] - sg.begin[h]) % 16 == 0;
    const int64_t units = al ? total / 16 : total;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((units + 255) / 256, 8192));
    if (al)
      hipLaunchKernelGGL(k_copy_segs<16>, dim3(grid), dim3(256), 0, s, sg, recv);
    else
      hipLaunchKernelGGL(k_copy_segs<1>, dim3(grid), dim3(256), 0, s, sg, recv);
    return hipGetLastError() == hipSuccess ? 0 : fail("local comm: copy kernel launch failed");
  }
  int grow(size_t bytes) {
    if (bytes <= tmp_bytes) return 0;
    if (tmp) (void)hipFree(tmp);
    tmp = nullptr;
    tmp_bytes = 0;
    if (hipMalloc(&tmp, bytes) != hipSuccess) return fail("local comm: scratch allocation failed");
    tmp_bytes = bytes;
    return 0;
  }
  // tmp[h*bytes ..] = rank h's send, for every h. On return every rank has
  // finished reading every send buffer, so recv (which may alias send) can
  // be written.
  int gather(const void* send, size_t bytes, hipStream_t s) {
    if (grow(bytes * world)) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return fail("local comm: stream sync failed");
    g->ptr[rank] = send;
    if (!g->barrier()) return fail("local comm: barrier timeout (a rank failed or diverged)");
    for (int h = 0; h < world; ++h)
      if (hipMemcpyPeerAsync(static_cast<char*>(tmp) + (size_t)h * bytes, device, g->ptr[h], g->dev[h], bytes, s) !=
          hipSuccess)
        return fail("local comm: peer copy failed");
    if (hipStreamSynchronize(s) != hipSuccess) return fail("local comm: stream sync failed");
    if (!g->barrier()) return fail("local comm: barrier timeout (a rank failed or diverged)");
    return 0;
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (bytes == 0) return 0;
    if (direct()) {
      // straight into recv: no rank reads it (a send aliasing recv's own
      // block gets its own bytes back)
      if (sync(s)) return -1;
      g->ptr[rank] = send;
      if (meet()) return -1;
      Segs sg{};
      sg.n = world;
      for (int h = 0; h < world; ++h) {
        sg.src[h] = static_cast<const char*>(g->ptr[h]);
        sg.dst[h] = (int64_t)h * (int64_t)bytes;
        sg.begin[h + 1] = sg.begin[h] + (int64_t)bytes;
      }
      if (copy_segs(sg, static_cast<char*>(recv), s) || sync(s) || meet()) return -1;
      return 0;
    }
    if (gather(send, bytes, s)) return -1;
    if (hipMemcpyAsync(recv, tmp, bytes * world, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return fail("local comm: copy failed");
    return 0;
  }
  template <typename T>
  void reduce(GhROp op, size_t count, void* recv, hipStream_t s) {
    const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, 4096);
    if (op == GH_OP_SUM)
      hipLaunchKernelGGL((k_reduce<T, GH_OP_SUM>), dim3(grid), dim3(256), 0, s, static_cast<const T*>(tmp), world,
                         count, static_cast<T*>(recv));
    else
      hipLaunchKernelGGL((k_reduce<T, GH_OP_MAX>), dim3(grid), dim3(256), 0, s, static_cast<const T*>(tmp), world,
                         count, static_cast<T*>(recv));
  }
  int share(const void* mine, hipStream_t s, const void** all) override {
    if (!direct()) return 1;
    if (sync(s)) return -1;
    g->ptr[rank] = mine;
    if (meet()) return -1;
    for (int h = 0; h < world; ++h) all[h] = g->ptr[h];
    return 0;
  }
  int share_done(hipStream_t s) override { return (sync(s) || meet()) ? -1 : 0; }
  // every rank publishes its send buffer and counts; each copies the blocks
  // addressed to it straight from the peers' buffers
  int alltoallv(const void* send, const size_t* sendbytes, void* recv, const size_t* recvbytes,
                hipStream_t s, const size_t* recvdispl) override {
    if (hipStreamSynchronize(s) != hipSuccess) return fail("local comm: stream sync failed");
    g->ptr[rank] = send;
    g->counts[rank] = sendbytes;
    if (!g->barrier()) return fail("local comm: barrier timeout (a rank failed or diverged)");
    if (direct()) {  // one copy kernel over the blocks addressed to this rank
      Segs sg{};
      size_t ro = 0;
      for (int h = 0; h < world; ++h) {
        size_t off = 0;
        for (int r = 0; r < rank; ++r) off += g->counts[h][r];
        const size_t bytes = g->counts[h][rank];
        if (bytes != recvbytes[h]) {
          g->barrier();
          return fail("local comm: alltoallv counts disagree");
        }
        sg.src[sg.n] = static_cast<const char*>(g->ptr[h]) + off;
        sg.dst[sg.n] = (int64_t)(recvdispl ? recvdispl[h] : ro);
        sg.begin[sg.n + 1] = sg.begin[sg.n] + (int64_t)bytes;
        sg.n++;
        ro += bytes;
      }
      if (copy_segs(sg, static_cast<char*>(recv), s) || sync(s) || meet()) return -1;
      return 0;
    }
    size_t ro = 0;
    for (int h = 0; h < world; ++h) {
      size_t off = 0;
      for (int r = 0; r < rank; ++r) off += g->counts[h][r];
      const size_t bytes = g->counts[h][rank];
      if (bytes != recvbytes[h]) {
        g->barrier();
        return fail("local comm: alltoallv counts disagree");
      }
      const size_t at = recvdispl ? recvdispl[h] : ro;
      if (bytes && hipMemcpyPeerAsync(static_cast<char*>(recv) + at, device, static_cast<const char*>(g->ptr[h]) + off,
                                      g->dev[h], bytes, s) != hipSuccess)
        return fail("local comm: peer copy failed");
      ro += bytes;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return fail("local comm: stream sync failed");
    if (!g->barrier()) return fail("local comm: barrier timeout (a rank failed or diverged)");
    return 0;
  }
  template <typename T>
  void reduce_ptrs(GhROp op, size_t count, T* out, hipStream_t s) {
    Ptrs ps{};
    for (int h = 0; h < world; ++h) ps.p[h] = g->ptr[h];
    const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, 4096);
    if (op == GH_OP_SUM)
      hipLaunchKernelGGL((k_reduce_ptrs<T, GH_OP_SUM>), dim3(grid), dim3(256), 0, s, ps, world, count, out);
    else
      hipLaunchKernelGGL((k_reduce_ptrs<T, GH_OP_MAX>), dim3(grid), dim3(256), 0, s, ps, world, count, out);
  }
  int allreduce(const void* send, void* recv, size_t count, GhDType dt, GhROp op, hipStream_t s) override {
    if (count == 0) return 0;
    if (direct()) {
      // one kernel reads every rank's send; in place (send == recv) through
      // tmp, as the other ranks may still be reading this send
      const size_t bytes = count * gh_dtype_size(dt);
      const bool inplace = send == recv;
      if ((inplace && grow(bytes)) || sync(s)) return -1;
      g->ptr[rank] = send;
      if (meet()) return -1;
      void* out = inplace ? tmp : recv;
      if (dt == GH_DT_U8)
        reduce_ptrs<uint8_t>(op, count, static_cast<uint8_t*>(out), s);
      else if (dt == GH_DT_I32)
        reduce_ptrs<int32_t>(op, count, static_cast<int32_t*>(out), s);
      else
        reduce_ptrs<unsigned long long>(op, count, static_cast<unsigned long long*>(out), s);
      if (hipGetLastError() != hipSuccess) return fail("local comm: reduce kernel launch failed");
      if (sync(s) || meet()) return -1;
      if (inplace && hipMemcpyAsync(recv, tmp, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return fail("local comm: copy failed");
      return 0;
    }
    if (gather(send, count * gh_dtype_size(dt), s)) return -1;
    if (dt == GH_DT_U8)
      reduce<uint8_t>(op, count, recv, s);
    else if (dt == GH_DT_I32)
      reduce<int32_t>(op, count, recv, s);
    else
      reduce<unsigned long long>(op, count, recv, s);
    return hipGetLastError() == hipSuccess ? 0 : fail("local comm: reduce kernel launch failed");
  }
};

}  // namespace

GhComm* gh_comm_single() { return new SingleComm(); }

int gh_comm_rccl_unique_id(uint8_t* id, std::string* err) {
  const RcclApi& a = rccl_api();
  if (!a.ok) {
    *err = a.load_err;
    return -1;
  }
  ncclUniqueId u;
  const ncclResult_t r = a.get_unique_id(&u);
  if (r != ncclSuccess) {
    *err = std::string("ncclGetUniqueId: ") + a.error_string(r);
    return -1;
  }
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

GhComm* gh_comm_rccl(int rank, int world, const uint8_t* id, std::string* err) {
  const RcclApi& a = rccl_api();
  if (!a.ok) {
    *err = a.load_err;
    return nullptr;
  }
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  RcclComm* c = new RcclComm();
  c->api = &a;
  c->rank = rank;
  c->world = world;
  const ncclResult_t r = a.comm_init_rank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    *err = std::string("ncclCommInitRank: ") + a.error_string(r);
    c->comm = nullptr;
    delete c;
    return nullptr;
  }
  return c;
}

GhComm* gh_comm_local(int rank, int world, const uint8_t* key, int device, std::string* err) {
  const std::string k(reinterpret_cast<const char*>(key), strnlen(reinterpret_cast<const char*>(key), 128));
  std::shared_ptr<LocalGroup> g;
  {
    std::lock_guard<std::mutex> l(g_groups_m);
    for (auto it = g_groups.begin(); it != g_groups.end();)
      it = it->second.expired() ? g_groups.erase(it) : std::next(it);
    auto it = g_groups.find(k);
    if (it != g_groups.end()) g = it->second.lock();
    if (!g) {
      g = std::make_shared<LocalGroup>(world);
      g_groups[k] = g;
    }
    if (g->world != world) {
      *err = "local comm: world size differs from the group's";
      return nullptr;
    }
    g->dev[rank] = device;
  }
  LocalComm* c = new LocalComm();
  c->g = g;
  c->rank = rank;
  c->world = world;
  c->device = device;
  return c;
}
