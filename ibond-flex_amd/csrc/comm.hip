// Ciphertext-shard all-gather over RCCL (xGMI), C ABI (include/flexpai.h pai_comm_*, pai_allgather_*).
//
// The shards of a sharded encryption (bench.py configs[3]/[4]) are reassembled on every
// rank by one all-gather of the ciphertext words and one of the exponents, grouped into one RCCL launch.
// Python callers can use torch.distributed (sharding.py); this entry point serves hosts that drive the
// engine through the C ABI alone (a cgo / JNI binding). RCCL is opened with dlopen on
// first use (RTLD_LOCAL | RTLD_DEEPBIND: a process may already hold another RCCL, e.g. PyTorch's), so
// libflexpai.so itself does not depend on it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "flexpai.h"

namespace fpai {
int set_error(int code, const char* msg);
}

struct pai_comm {
  ncclComm_t comm = nullptr;
  int world = 0, rank = 0, device = 0;
};

namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string why;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = getenv("FLEXPAI_RCCL_LIB");
    for (const char* name : {env, "/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"}) {
      if (!name) continue;
      r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
      if (r.h) break;
    }
    if (!r.h) {
      r.why = "RCCL not found (librccl.so.1)";
      return;
    }
    auto sym = [&](const char* s) { return dlsym(r.h, s); };
    r.get_unique_id = (decltype(r.get_unique_id))sym("ncclGetUniqueId");
    r.init_rank = (decltype(r.init_rank))sym("ncclCommInitRank");
    r.all_gather = (decltype(r.all_gather))sym("ncclAllGather");
    r.group_start = (decltype(r.group_start))sym("ncclGroupStart");
    r.group_end = (decltype(r.group_end))sym("ncclGroupEnd");
    r.destroy = (decltype(r.destroy))sym("ncclCommDestroy");
    r.error_string = (decltype(r.error_string))sym("ncclGetErrorString");
    if (!r.get_unique_id || !r.init_rank || !r.all_gather || !r.group_start || !r.group_end || !r.destroy)
      r.why = "RCCL is missing a symbol";
  });
  return r;
}

int rccl_fail(ncclResult_t e, const char* what) {
  std::string m = std::string(what) + ": " + (rccl().error_string ? rccl().error_string(e) : "RCCL error");
  return fpai::set_error(PAI_ERR_HIP, m.c_str());
}

int ready() {
  Rccl& r = rccl();
  if (!r.why.empty()) return fpai::set_error(PAI_ERR_HIP, r.why.c_str());
  return 0;
}

}  // namespace

extern "C" {

int pai_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return fpai::set_error(PAI_ERR_ARG, "pai_comm_unique_id: null buffer");
  if (int rc = ready()) return rc;
  ncclUniqueId id;
  if (ncclResult_t e = rccl().get_unique_id(&id)) return rccl_fail(e, "ncclGetUniqueId");
  std::memcpy(id_out, id.internal, PAI_COMM_ID_BYTES);
  return 0;
}

int pai_comm_create(const uint8_t* id, int world, int rank, int device, pai_comm** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return fpai::set_error(PAI_ERR_ARG, "pai_comm_create: bad arguments");
  *out = nullptr;
  if (int rc = ready()) return rc;
  if (hipSetDevice(device) != hipSuccess) return fpai::set_error(PAI_ERR_HIP, "pai_comm_create: hipSetDevice failed");
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, PAI_COMM_ID_BYTES);
  pai_comm* c = new pai_comm;
  c->world = world;
  c->rank = rank;
  c->device = device;
  if (ncclResult_t e = rccl().init_rank(&c->comm, world, uid, rank)) {
    delete c;
    return rccl_fail(e, "ncclCommInitRank");
  }
  *out = c;
  return 0;
}

void pai_comm_destroy(pai_comm* c) {
  if (!c) return;
  if (c->comm) (void)rccl().destroy(c->comm);
  delete c;
}

int pai_allgather_dev(pai_comm* c, const void* d_send, size_t bytes_per_rank, void* d_recv, void* stream) {
  if (!c || (!d_send && bytes_per_rank) || (!d_recv && bytes_per_rank))
    return fpai::set_error(PAI_ERR_ARG, "pai_allgather_dev: bad arguments");
  if (bytes_per_rank == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return fpai::set_error(PAI_ERR_HIP, "hipSetDevice failed");
  if (ncclResult_t e = rccl().all_gather(d_send, d_recv, bytes_per_rank, ncclUint8, c->comm, (hipStream_t)stream))
    return rccl_fail(e, "ncclAllGather");
  return 0;
}

int pai_allgather_shards_dev(pai_comm* c, const uint32_t* d_ct, const int32_t* d_exp, size_t n_per_rank, int ct_words,
                             uint32_t* d_ct_all, int32_t* d_exp_all, void* stream) {
  if (!c || ct_words < 1 || (n_per_rank && (!d_ct || !d_exp || !d_ct_all || !d_exp_all)))
    return fpai::set_error(PAI_ERR_ARG, "pai_allgather_shards_dev: bad arguments");
  if (n_per_rank == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return fpai::set_error(PAI_ERR_HIP, "hipSetDevice failed");
  Rccl& r = rccl();
  hipStream_t st = (hipStream_t)stream;
  if (ncclResult_t e = r.group_start()) return rccl_fail(e, "ncclGroupStart");
  ncclResult_t e1 = r.all_gather(d_ct, d_ct_all, n_per_rank * (size_t)ct_words, ncclUint32, c->comm, st);
  ncclResult_t e2 = r.all_gather(d_exp, d_exp_all, n_per_rank, ncclInt32, c->comm, st);
  ncclResult_t e3 = r.group_end();
  if (e1) return rccl_fail(e1, "ncclAllGather (ciphertexts)");
  if (e2) return rccl_fail(e2, "ncclAllGather (exponents)");
  if (e3) return rccl_fail(e3, "ncclGroupEnd");
  return 0;
}

}  // extern "C"
