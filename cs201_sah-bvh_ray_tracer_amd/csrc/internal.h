// Internal helpers shared by the host translation units of libmirt.so.
#pragma once
#include <cstdarg>
#include <cstdio>

#include "../../include/mirt.h"

namespace mirt {

// Thread-local last error (mirt_last_error()).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Shard geometry of mirt_frame_desc (csrc/shard.h): row r of the compacted
// shard is image row y = shard_block(shard, r / rb) * rb + r % rb.
int shard_row_count(const mirt_frame_desc* fd);
bool frame_desc_valid(const mirt_frame_desc* fd);

// A well-formed flat pre-order tree (mirt_node): root skip == nn; every skip
// in (i, nn]; leaves skip to i + 1 and index spheres in [sphere_lo,
// num_spheres] (num_spheres: the never-hit sentinel); the empty flag only on
// leaves; every inner node's two subtrees [i+1, r) and [r, skip) nest inside
// it. MIRT_OK or MIRT_E_INVALID with the message prefixed by `fn`.
int validate_flat(const mirt_node* nd, int nn, int num_spheres, int sphere_lo, const char* fn);

// render.hip: the frame of mirt_render_frame up to its D2H copy, enqueued on
// the ctx's own stream into d_out (fd->samples slabs of the shard; the ctx's
// own buffer when null) with the ctx's (possibly shared) accumulation buffer;
// *d_display = the slab holding the display after the last frame.
// independent (fd->samples > 1, !fd->accumulate): the samples are successive
// FRESH frames (main.c:358-374 each), left raw in their slabs, the last one
// folded into the accumulation buffer as a fresh frame; otherwise they fold in
// order (a frame of several samples / the accumulating display loop).
int enqueue_frame_device(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, uint32_t* d_out,
                         uint32_t** d_display, const char* fn, bool independent = false);
int ctx_device(const mirt_ctx* c);
// [p, p + bytes) is ONE page-locked host range (mirt_host_alloc /
// mirt_host_register): copies into it are DMA, asynchronous to the host.
bool host_page_locked(const void* p, size_t bytes);
uint32_t* host_device_ptr(const void* p, size_t bytes);
int accum_settle(mirt_ctx* c);
void pinned_add(const void* p, size_t bytes);   // mirt_host_alloc / mirt_host_register ranges
void pinned_remove(const void* p);

}  // namespace mirt
