// Internal helpers shared by the host translation units of libmirt.so.
#pragma once
#include <cstdarg>
#include <cstdio>

#include "../../include/mirt.h"

namespace mirt {

// Thread-local last error (mirt_last_error()).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Shard geometry of mirt_frame_desc: row r of the compacted shard is image
// row y = ((r / rb) * num_shards + shard) * rb + r % rb.
int shard_row_count(const mirt_frame_desc* fd);
bool frame_desc_valid(const mirt_frame_desc* fd);

}  // namespace mirt
