// comm.cpp — RCCL over xGMI for the §8e frame reduce (SURVEY §8b lists ptgs_reduce_radiance): the
// path tracer shards samples across GPUs and sums the RGBA32F radiance buffers; the 3DGS tile-row
// shard gathers disjoint partial frames with the same reduce. The reference has no multi-GPU path.
//
// RCCL is resolved at run time (dlopen of librccl.so.1, reusing a copy the process already loaded,
// e.g. PyTorch's) so libptgs loads on machines without it; the entry points then fail with
// PTGS_EHIP. One communicator per context, created from a 128-byte unique id that one rank makes
// (ptgs_comm_unique_id) and the caller distributes (any out-of-band channel).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and enums only; the symbols are resolved with dlsym

#include <cstring>

#include "../../include/ptgs/ptgs.h"
#include "comm.h"

namespace {

static_assert(sizeof(ncclUniqueId) == PTGS_COMM_ID_BYTES, "ncclUniqueId size");
typedef ncclComm_t nccl_comm_t;
typedef ncclUniqueId nccl_unique_id_t;

struct Rccl {
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(nccl_unique_id_t*) = nullptr;
  ncclResult_t (*comm_init_rank)(nccl_comm_t*, int, nccl_unique_id_t, int) = nullptr;
  ncclResult_t (*comm_destroy)(nccl_comm_t) = nullptr;
  ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, nccl_comm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, nccl_comm_t, hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, nccl_comm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, nccl_comm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

Rccl& rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r;
  tried = true;
  const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
  for (const char* n : names) {
    r.so = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    if (!r.so) r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (r.so) break;
  }
  if (!r.so) return r;
  r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.so, "ncclGetUniqueId");
  r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.so, "ncclCommInitRank");
  r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.so, "ncclCommDestroy");
  r.reduce = (decltype(r.reduce))dlsym(r.so, "ncclReduce");
  r.all_reduce = (decltype(r.all_reduce))dlsym(r.so, "ncclAllReduce");
  r.error_string = (decltype(r.error_string))dlsym(r.so, "ncclGetErrorString");
  r.send = (decltype(r.send))dlsym(r.so, "ncclSend");
  r.recv = (decltype(r.recv))dlsym(r.so, "ncclRecv");
  r.group_start = (decltype(r.group_start))dlsym(r.so, "ncclGroupStart");
  r.group_end = (decltype(r.group_end))dlsym(r.so, "ncclGroupEnd");
  r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.reduce && r.all_reduce && r.error_string &&
         r.send && r.recv && r.group_start && r.group_end;
  return r;
}

}  // namespace

namespace ptgs {

const char* comm_error(int code) {
  Rccl& r = rccl();
  return (r.ok && r.error_string) ? r.error_string((ncclResult_t)code) : "RCCL unavailable";
}

bool comm_available() { return rccl().ok; }

int comm_unique_id(uint8_t* id) {
  Rccl& r = rccl();
  if (!r.ok) return -1;
  nccl_unique_id_t u;
  ncclResult_t e = r.get_unique_id(&u);
  if (e != ncclSuccess) return (int)e;
  std::memcpy(id, u.internal, PTGS_COMM_ID_BYTES);
  return 0;
}

int comm_create(const uint8_t* id, int nranks, int rank, void** comm) {
  Rccl& r = rccl();
  if (!r.ok) return -1;
  nccl_unique_id_t u;
  std::memcpy(u.internal, id, PTGS_COMM_ID_BYTES);
  nccl_comm_t c = nullptr;
  ncclResult_t e = r.comm_init_rank(&c, nranks, u, rank);
  if (e != ncclSuccess) return (int)e;
  *comm = c;
  return 0;
}

int comm_destroy(void* comm) {
  Rccl& r = rccl();
  if (!r.ok || !comm) return 0;
  return (int)r.comm_destroy((nccl_comm_t)comm);
}

int comm_reduce_sum(void* comm, float* buf, size_t n, int root, hipStream_t s) {
  Rccl& r = rccl();
  if (!r.ok) return -1;
  return (int)r.reduce(buf, buf, n, ncclFloat32, ncclSum, root, (nccl_comm_t)comm, s);
}

int comm_allreduce_sum(void* comm, float* buf, size_t n, hipStream_t s) {
  Rccl& r = rccl();
  if (!r.ok) return -1;
  return (int)r.all_reduce(buf, buf, n, ncclFloat32, ncclSum, (nccl_comm_t)comm, s);
}

// Every rank's own rows [range[2 g], range[2 g + 1]) of a row-major buffer (row_floats floats per
// row) to the same rows of root's buffer: one ncclSend per rank, root posts the matching ncclRecv's,
// all in one group (the disjoint tile-row shards of the splat: W*H*16/G bytes per rank instead of a
// full-frame reduce).
int comm_gather_rows(void* comm, float* buf, size_t row_floats, const uint32_t* range, int nranks, int rank, int root,
                     hipStream_t s) {
  Rccl& r = rccl();
  if (!r.ok) return -1;
  nccl_comm_t c = (nccl_comm_t)comm;
  ncclResult_t e = r.group_start();
  if (e != ncclSuccess) return (int)e;
  for (int g = 0; g < nranks && e == ncclSuccess; ++g) {
    const size_t off = (size_t)range[2 * g] * row_floats;
    const size_t n = range[2 * g + 1] > range[2 * g] ? (size_t)(range[2 * g + 1] - range[2 * g]) * row_floats : 0;
    if (g == root || n == 0) continue;
    if (rank == g) e = r.send(buf + off, n, ncclFloat32, root, c, s);
    else if (rank == root) e = r.recv(buf + off, n, ncclFloat32, g, c, s);
  }
  ncclResult_t e2 = r.group_end();
  return (int)(e != ncclSuccess ? e : e2);
}

// Reduce-scatter by rows: every rank g receives, in its own buffer's rows [range[2 g], range[2 g + 1]),
// the SUM over the ranks of those rows (the other rows are left as they were): one ncclReduce per
// rank's slice (root g, in place), all in one group so they proceed together. Each rank sends about
// one frame ((G-1)/G of it) instead of an all-reduce's two; the C5 hybrid needs the path-traced
// radiance only under the tile rows it composites.
int comm_reduce_rows(void* comm, float* buf, size_t row_floats, const uint32_t* range, int nranks, hipStream_t s) {
  Rccl& r = rccl();
  if (!r.ok) return -1;
  nccl_comm_t c = (nccl_comm_t)comm;
  ncclResult_t e = r.group_start();
  if (e != ncclSuccess) return (int)e;
  for (int g = 0; g < nranks && e == ncclSuccess; ++g) {
    if (range[2 * g + 1] <= range[2 * g]) continue;
    float* p = buf + (size_t)range[2 * g] * row_floats;
    e = r.reduce(p, p, (size_t)(range[2 * g + 1] - range[2 * g]) * row_floats, ncclFloat32, ncclSum, g, c, s);
  }
  ncclResult_t e2 = r.group_end();
  return (int)(e != ncclSuccess ? e : e2);
}

}  // namespace ptgs
