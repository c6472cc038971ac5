// The data-parallel gather of the sampling harness as a C-ABI collective over RCCL (include/dm_hip.h
// dm_comm_*). It replaces accelerate's `accelerator.gather(samples)` of the finished fold (reference
// scripts/sample_uncond.py:190, scripts/sample_cfg.py:177): each rank contributes its [bspp, C, H, W] fold
// and receives the world's folds concatenated in rank order -- one all-gather per fold, no collective
// on the denoising path itself.
//
// RCCL is resolved at dm_comm_init time with dlopen("librccl.so.1") instead of a link-time dependency:
// the library then loads on hosts without RCCL (the CPU test container), and inside a PyTorch-ROCm process
// the soname resolves to the RCCL torch already mapped, so the process holds one RCCL. The bootstrap is
// RCCL's own: rank 0 draws the 128-byte unique id (dm_comm_unique_id), the caller moves it to the other
// ranks by any means (the harness uses the torch.distributed store it already has), every rank calls
// dm_comm_init on its own device.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <cstring>
#include <string>
#include "dm_common.h"

namespace dm {
namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
  bool ok = false;
};

template <class F>
bool sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl t;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return t;
    t.ok = sym(h, "ncclGetUniqueId", t.get_unique_id) && sym(h, "ncclCommInitRank", t.init_rank) &&
           sym(h, "ncclAllGather", t.all_gather) && sym(h, "ncclCommDestroy", t.destroy) &&
           sym(h, "ncclGetErrorString", t.error_string) && sym(h, "ncclCommCount", t.count) &&
           sym(h, "ncclCommUserRank", t.user_rank);
    return t;
  }();
  return r;
}

int need_rccl() {
  if (rccl().ok) return DM_OK;
  const char* e = dlerror();
  set_error(std::string("RCCL (librccl.so.1) could not be loaded: ") + (e ? e : "missing symbols"));
  return DM_ERR_UNSUPPORTED;
}

int rccl_error(ncclResult_t r, const char* what) {
  set_error(std::string(what) + ": " + rccl().error_string(r));
  return DM_ERR_HIP;
}

struct Comm {
  ncclComm_t comm;
  int nranks, rank, device;
};

}  // namespace
}  // namespace dm

static_assert(sizeof(ncclUniqueId) == DM_COMM_UID_BYTES, "RCCL unique id size");

extern "C" int dm_comm_unique_id(void* uid) {
  if (!uid) { dm::set_error("null unique-id buffer"); return DM_ERR_ARG; }
  if (int rc = dm::need_rccl()) return rc;
  ncclUniqueId id;
  if (ncclResult_t r = dm::rccl().get_unique_id(&id)) return dm::rccl_error(r, "ncclGetUniqueId");
  std::memcpy(uid, &id, sizeof(id));
  return DM_OK;
}

extern "C" int dm_comm_init(const void* uid, int nranks, int rank, dm_comm** comm) {
  if (!uid || !comm) { dm::set_error("null argument"); return DM_ERR_ARG; }
  if (nranks <= 0 || rank < 0 || rank >= nranks) { dm::set_error("rank must lie in [0, nranks)"); return DM_ERR_ARG; }
  *comm = nullptr;
  if (int rc = dm::need_rccl()) return rc;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { dm::set_error("hipGetDevice failed"); return DM_ERR_HIP; }
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  ncclComm_t c = nullptr;
  if (ncclResult_t r = dm::rccl().init_rank(&c, nranks, id, rank)) return dm::rccl_error(r, "ncclCommInitRank");
  *comm = reinterpret_cast<dm_comm*>(new dm::Comm{c, nranks, rank, dev});
  return DM_OK;
}

extern "C" int dm_comm_info(const dm_comm* comm, int* nranks, int* rank, int* device) {
  if (!comm) { dm::set_error("null communicator"); return DM_ERR_ARG; }
  const dm::Comm* c = reinterpret_cast<const dm::Comm*>(comm);
  int n = 0, r = 0;
  if (ncclResult_t e = dm::rccl().count(c->comm, &n)) return dm::rccl_error(e, "ncclCommCount");
  if (ncclResult_t e = dm::rccl().user_rank(c->comm, &r)) return dm::rccl_error(e, "ncclCommUserRank");
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (device) *device = c->device;
  return DM_OK;
}

extern "C" int dm_allgather_f32(dm_comm* comm, const float* send, float* recv, int64_t count, void* stream) {
  if (!comm) { dm::set_error("null communicator"); return DM_ERR_ARG; }
  if (count < 0) { dm::set_error("negative element count"); return DM_ERR_ARG; }
  if (count == 0) return DM_OK;
  if (!send || !recv) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  dm::Comm* c = reinterpret_cast<dm::Comm*>(comm);
  // recv holds nranks x count floats; send may alias recv's own slot (in-place all-gather)
  if (ncclResult_t r = dm::rccl().all_gather(send, recv, (size_t)count, ncclFloat32, c->comm, (hipStream_t)stream))
    return dm::rccl_error(r, "ncclAllGather");
  return DM_OK;
}

extern "C" void dm_comm_destroy(dm_comm* comm) {
  if (!comm) return;
  dm::Comm* c = reinterpret_cast<dm::Comm*>(comm);
  dm::rccl().destroy(c->comm);
  delete c;
}
