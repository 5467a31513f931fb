// hj_launch.h — host-callable launchers of the gfx950 kernels (implemented in
// hj_kernels.hip). Every launcher is asynchronous on `stream` and returns the
// hipError_t of the launch.
#pragma once
#include <hip/hip_runtime.h>
#include "hj_device.h"

namespace dfp {

// ---- build ---------------------------------------------------------------
hipError_t launch_insert(int key_bytes, const Segment* d_segs, int nseg, int64_t total,
                         Bucket* tbl, uint32_t nbuckets, uint64_t* row_ids,
                         uint2* duprows, uint32_t* dupslots, BuildCounters* ctr,
                         int grid, hipStream_t s);
hipError_t launch_dup_passes(Bucket* tbl, uint32_t nbuckets, const uint2* duprows,
                             const uint32_t* dupslots, DupDir* dir, uint32_t* dup_rows,
                             uint32_t* big, BuildCounters* ctr, int grid, hipStream_t s);

hipError_t launch_dup_big(Bucket* tbl, uint32_t nbuckets, const DupDir* dir, uint32_t* dup_rows,
                          const uint32_t* big, const BuildCounters* ctr, const Segment* segs,
                          int nseg, int64_t total, int key_bytes, int grid, hipStream_t s);

// ---- probe ---------------------------------------------------------------
int64_t probe_tiles(int64_t n);
hipError_t launch_probe(int key_bytes, const Bucket* tbl, uint32_t nbuckets,
                        const uint32_t* dup_rows, const uint64_t* row_ids,
                        const void* keys, const uint8_t* valid, int64_t voff,
                        const uint32_t* probe_ids, int64_t n, uint64_t* out_b,
                        uint32_t* out_p, int64_t cap, int64_t* d_total,
                        unsigned long long* status, unsigned int* ticket,
                        hipStream_t s);

// ---- table queries -------------------------------------------------------
hipError_t launch_table_stats(const Bucket* tbl, uint32_t nbuckets,
                              unsigned long long* out /* [4]: distinct, dupkeys, duprows, maxrows */,
                              hipStream_t s);
hipError_t launch_chain_links(const Bucket* tbl, uint32_t nbuckets, const uint32_t* dup_rows,
                              int64_t* prev, int64_t nrows, hipStream_t s);

// ---- multi-GPU radix partition -------------------------------------------
hipError_t launch_radix_partition(int key_bytes, const void* keys, const uint8_t* valid,
                                  int64_t voff, const uint64_t* ids, uint64_t id_base,
                                  int64_t n, int nparts, void* out_keys, uint64_t* out_ids,
                                  int64_t* counts, void* workspace, hipStream_t s);
int64_t radix_partition_workspace(int64_t n, int nparts);

// ---- generators ----------------------------------------------------------
hipError_t launch_gen_perm(int64_t* out, int64_t n, int64_t mul, int64_t range, hipStream_t s);
hipError_t launch_gen_uniform(int64_t* out, int64_t n, uint64_t seed, int64_t range,
                              hipStream_t s);

}  // namespace dfp
