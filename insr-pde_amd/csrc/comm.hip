// comm.hip -- the data-parallel collective of the training step behind the C ABI: one
// sum all-reduce of the flat gradient buffer (+ loss scalars) per optimiser step over RCCL
// (xGMI inside a node).  This is what the reference's DDP-style scaling needs from a
// non-Python host (SURVEY.md §8 b: insr_comm_init / insr_allreduce_sum); the Python
// package uses torch.distributed (backend "nccl" = RCCL) for the same single collective.
//
// RCCL is resolved at run time (dlopen "librccl.so.1"): inside a PyTorch process that
// returns the RCCL torch already loaded (same soname), so one copy of the library
// serves both; elsewhere the ROCm one.  No link-time dependency.
#include <dlfcn.h>

#include <cstring>

#include "jet_common.hpp"

namespace insr {

typedef struct {
  char internal[128];
} RcclId;
typedef int (*GetUniqueIdFn)(RcclId*);
typedef int (*CommInitRankFn)(void** comm, int nranks, RcclId id, int rank);
typedef int (*AllReduceFn)(const void*, void*, size_t, int datatype, int op, void* comm, hipStream_t);
typedef int (*CommDestroyFn)(void*);

constexpr int kRcclFloat32 = 7, kRcclSum = 0;  // ncclFloat32, ncclSum (rccl.h)

struct Rccl {
  bool tried = false, ok = false;
  GetUniqueIdFn get_id = nullptr;
  CommInitRankFn init = nullptr;
  AllReduceFn allreduce = nullptr;
  CommDestroyFn destroy = nullptr;
};

static Rccl& rccl() {
  static Rccl r;
  if (!r.tried) {
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h) {
      r.get_id = (GetUniqueIdFn)dlsym(h, "ncclGetUniqueId");
      r.init = (CommInitRankFn)dlsym(h, "ncclCommInitRank");
      r.allreduce = (AllReduceFn)dlsym(h, "ncclAllReduce");
      r.destroy = (CommDestroyFn)dlsym(h, "ncclCommDestroy");
      r.ok = r.get_id && r.init && r.allreduce && r.destroy;
    }
  }
  return r;
}

}  // namespace insr

using namespace insr;

extern "C" {

int insr_comm_available(void) { return rccl().ok ? 1 : 0; }

long insr_comm_id_bytes(void) { return (long)sizeof(RcclId); }

int insr_comm_unique_id(void* id_out) {
  Rccl& r = rccl();
  if (!r.ok) return INSR_ENOCOMM;
  if (!id_out) return INSR_EINVAL;
  RcclId id;
  const int rc = r.get_id(&id);
  if (rc) return INSR_ECOMM_BASE + rc;
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}

int insr_comm_init(void** comm, int rank, int world, const void* id) {
  Rccl& r = rccl();
  if (!r.ok) return INSR_ENOCOMM;
  if (!comm || !id || world < 1 || rank < 0 || rank >= world) return INSR_EINVAL;
  RcclId cid;
  std::memcpy(&cid, id, sizeof(cid));
  const int rc = r.init(comm, world, cid, rank);
  return rc ? INSR_ECOMM_BASE + rc : 0;
}

int insr_comm_allreduce_sum(void* comm, float* buf, long count, void* stream) {
  Rccl& r = rccl();
  if (!r.ok) return INSR_ENOCOMM;
  if (!comm || count < 0 || (count > 0 && !buf)) return INSR_EINVAL;
  if (count == 0) return 0;
  const int rc = r.allreduce(buf, buf, (size_t)count, kRcclFloat32, kRcclSum, comm, (hipStream_t)stream);
  return rc ? INSR_ECOMM_BASE + rc : 0;
}

int insr_comm_destroy(void* comm) {
  Rccl& r = rccl();
  if (!r.ok) return INSR_ENOCOMM;
  if (!comm) return INSR_EINVAL;
  const int rc = r.destroy(comm);
  return rc ? INSR_ECOMM_BASE + rc : 0;
}

}  // extern "C"
