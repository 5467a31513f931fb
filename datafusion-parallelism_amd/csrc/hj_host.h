// hj_host.h — internal hooks of the host layer (hj_api.cpp) for the other host
// translation units of the library (hj_dist.cpp). Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <string>

#include "../../include/hj.h"

namespace dfp {
namespace host {

// sets the thread-local message hj_last_error() returns; -> st
hj_status set_error(hj_status st, const std::string& msg);
// a block of the library's caching device allocator (nullptr on failure) / back to it
// (only once no queued work uses it)
void* dev_block(int dev, size_t bytes);
void free_block(int dev, void* p, size_t bytes);
// the table frees `p` (a dev_block) when it is freed, after its build and probes
void table_adopt_block(hj_table* t, int dev, void* p, size_t bytes);
// the table frees `other` when it is freed (a piece whose arrays were copied out)
void table_adopt_table(hj_table* t, hj_table* other);
// the table's build time runs from `ev` (a timing event the caller recorded where the
// work the table stands for began, e.g. a multi-GPU build side); the table owns it
void table_set_start_event(hj_table* t, hipEvent_t ev);

}  // namespace host
}  // namespace dfp
