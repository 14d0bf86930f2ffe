// pmvs_rccl.cpp -- native RCCL communicator for the sharded expansion.
//
// One process per GPU.  Rank 0 creates an RCCL unique id (pmvs_rccl_unique_id), the launcher
// hands its 128 bytes to every rank by any channel (bench.py: torch.distributed broadcast), and
// every rank builds its communicator with pmvs_rccl_create on its own device.  The context then
// serves two exchanges of pmvs_expand_run:
//   * pmvs_rccl_allgather (a pmvs_allgather_fn): host buffers, for the 8-byte error headers;
//   * the device all-gather of each wave's refined records (pmvs_scene_set_shard_rccl): the
//     rank's status / patch range is packed on the device and ncclAllGather'ed on the scene's
//     stream straight into the other ranks' device buffers -- no host staging, no Python.
// librccl is opened at run time (dlopen "librccl.so.1"), so the product library loads on hosts
// without RCCL and only these entry points fail (PMVS_EUNSUPPORTED) there.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <mutex>

#include "../../include/pmvs_amd.h"

pmvs_status pmvs_io_fail(pmvs_status st, const char* fmt, ...);  // pmvs_api.cpp: sets pmvs_last_error

namespace {

// The few RCCL symbols used (rccl.h: ncclResult_t is an int enum, ncclComm_t an opaque pointer).
constexpr int kIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
struct UniqueId {
  char internal[kIdBytes];
};
typedef int (*GetUniqueIdFn)(UniqueId*);
typedef int (*CommInitRankFn)(void** comm, int nranks, UniqueId id, int rank);
typedef int (*AllGatherFn)(const void* send, void* recv, size_t count, int datatype, void* comm, hipStream_t stream);
typedef int (*CommDestroyFn)(void* comm);
typedef const char* (*GetErrorStringFn)(int);
constexpr int kNcclUint8 = 1;  // ncclUint8 (rccl.h: ncclInt8 = 0, ncclUint8 = 1)

struct Rccl {
  void* h = nullptr;
  GetUniqueIdFn get_id = nullptr;
  CommInitRankFn init_rank = nullptr;
  AllGatherFn all_gather = nullptr;
  CommDestroyFn destroy = nullptr;
  GetErrorStringFn err = nullptr;
  bool ok = false;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) return;
    r.get_id = reinterpret_cast<GetUniqueIdFn>(dlsym(r.h, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<CommInitRankFn>(dlsym(r.h, "ncclCommInitRank"));
    r.all_gather = reinterpret_cast<AllGatherFn>(dlsym(r.h, "ncclAllGather"));
    r.destroy = reinterpret_cast<CommDestroyFn>(dlsym(r.h, "ncclCommDestroy"));
    r.err = reinterpret_cast<GetErrorStringFn>(dlsym(r.h, "ncclGetErrorString"));
    r.ok = r.get_id && r.init_rank && r.all_gather && r.destroy;
  });
  return r;
}

}  // namespace

struct pmvs_rccl {
  int device = 0, rank = 0, world = 1;
  void* comm = nullptr;
  hipStream_t stream = nullptr;  // host-buffer exchanges
  void* dsend = nullptr;
  void* drecv = nullptr;
  size_t cap = 0;
};

pmvs_status pmvs_rccl_unique_id(uint8_t* id) {
  if (!id) return pmvs_io_fail(PMVS_EINVAL, "null id");
  Rccl& r = rccl();
  if (!r.ok) return pmvs_io_fail(PMVS_EUNSUPPORTED, "librccl.so.1 not available");
  UniqueId u;
  const int e = r.get_id(&u);
  if (e != 0) return pmvs_io_fail(PMVS_EDEVICE, "ncclGetUniqueId: %s", r.err ? r.err(e) : "error");
  std::memcpy(id, u.internal, kIdBytes);
  return PMVS_OK;
}

pmvs_status pmvs_rccl_create(int32_t device, int32_t rank, int32_t world, const uint8_t* id, pmvs_rccl** out) {
  if (!out || !id || world < 1 || rank < 0 || rank >= world) return pmvs_io_fail(PMVS_EINVAL, "invalid rccl arguments");
  *out = nullptr;
  Rccl& r = rccl();
  if (!r.ok) return pmvs_io_fail(PMVS_EUNSUPPORTED, "librccl.so.1 not available");
  if (hipSetDevice(device) != hipSuccess) return pmvs_io_fail(PMVS_EDEVICE, "hipSetDevice(%d)", device);
  auto* c = new pmvs_rccl();
  c->device = device;
  c->rank = rank;
  c->world = world;
  UniqueId u;
  std::memcpy(u.internal, id, kIdBytes);
  const int e = r.init_rank(&c->comm, world, u, rank);
  if (e != 0) {
    delete c;
    return pmvs_io_fail(PMVS_EDEVICE, "ncclCommInitRank(rank %d of %d): %s", rank, world, r.err ? r.err(e) : "error");
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    pmvs_rccl_destroy(c);
    return pmvs_io_fail(PMVS_EDEVICE, "stream creation failed");
  }
  *out = c;
  return PMVS_OK;
}

void pmvs_rccl_destroy(pmvs_rccl* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->comm) (void)rccl().destroy(c->comm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->dsend) (void)hipFree(c->dsend);
  if (c->drecv) (void)hipFree(c->drecv);
  delete c;
}

int pmvs_rccl_allgather_device(void* ctx, const void* dsend, int64_t bytes, void* drecv, void* stream) {
  auto* c = static_cast<pmvs_rccl*>(ctx);
  if (!c || bytes < 0) return -1;
  if (bytes == 0) return 0;
  const int e = rccl().all_gather(dsend, drecv, (size_t)bytes, kNcclUint8, c->comm, static_cast<hipStream_t>(stream));
  return e == 0 ? 0 : -1;
}

int pmvs_rccl_allgather(void* ctx, const void* send, int64_t bytes, void* recv) {
  auto* c = static_cast<pmvs_rccl*>(ctx);
  if (!c || bytes < 0) return -1;
  if (bytes == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -1;
  const size_t need = (size_t)bytes * (size_t)(c->world + 1);
  if (need > c->cap) {
    if (c->dsend) (void)hipFree(c->dsend);
    c->dsend = c->drecv = nullptr;
    c->cap = 0;
    if (hipMalloc(&c->dsend, (size_t)bytes * (c->world + 1) + 256) != hipSuccess) return -1;
    c->cap = need;
  }
  char* ds = static_cast<char*>(c->dsend);
  char* dr = ds + bytes;
  if (hipMemcpyAsync(ds, send, (size_t)bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return -1;
  if (pmvs_rccl_allgather_device(c, ds, bytes, dr, c->stream) != 0) return -1;
  if (hipMemcpyAsync(recv, dr, (size_t)bytes * c->world, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return -1;
  return hipStreamSynchronize(c->stream) == hipSuccess ? 0 : -1;
}
