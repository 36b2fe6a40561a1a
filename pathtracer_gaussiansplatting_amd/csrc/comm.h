// comm.h — RCCL binding used by the C-ABI's ptgs_comm_* / ptgs_*reduce_radiance (comm.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ptgs {

bool comm_available();
const char* comm_error(int code);
int comm_unique_id(uint8_t* id);  // PTGS_COMM_ID_BYTES bytes
int comm_create(const uint8_t* id, int nranks, int rank, void** comm);
int comm_destroy(void* comm);
int comm_reduce_sum(void* comm, float* buf, size_t n, int root, hipStream_t s);
int comm_allreduce_sum(void* comm, float* buf, size_t n, hipStream_t s);
int comm_gather_rows(void* comm, float* buf, size_t row_floats, const uint32_t* range, int nranks, int rank, int root,
                     hipStream_t s);
int comm_reduce_rows(void* comm, float* buf, size_t row_floats, const uint32_t* range, int nranks, hipStream_t s);

}  // namespace ptgs
