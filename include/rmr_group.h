/*
 * rmr_group.h — C ABI of librmr_group.so: the frame tile-partitioned over several GPUs of one node
 * from ONE host process (SURVEY §5 "one process with one HIP stream per GPU and ncclCommInitAll";
 * §8e: "the image is tile-partitioned across the GPUs ... with a single RCCL reduce of the per-tile
 * radiance accumulator").
 *
 * The reference renders from one process with one GL context (Program.cpp:92-100, Graphics::Init,
 * Graphics.cpp:263-312); a C++ integrator of the drop-in keeps that shape and gets every GPU of the
 * node through this group. (The Python multi-process path, raymarchrenderer_amd/multi_gpu.py over
 * torch.distributed, is the same partition and schedule with one process per GPU.)
 *
 * Partition and schedule (the same as multi_gpu.FrameRenderer):
 *   - the frame's tile_size x tile_size tiles (row-major over the image) are dealt round-robin to the
 *     members: member m of n renders tiles m, m + n, m + 2n, ... (rmr_group_partition);
 *   - every member renders its tiles into its own zeroed full-frame RGBA32F accumulator (zero
 *     outside its tiles), then ONE ncclReduce(SUM) per frame sums the members' frames onto member 0
 *     over xGMI; x + 0 = x, so the frame is bitwise the one-GPU image;
 *   - each member holds two rmr contexts on two HIP streams with a frame buffer each; frames
 *     alternate between them, so frame f's reduce and its persistent kernel's drain overlap frame
 *     f + 1's render, and each trace launch leaves 64 workgroups free (rmr_set_grid_reserve) for the
 *     other context's fold, zeroing and reduce.
 * RCCL is loaded by this library only (librmr.so, the single-GPU drop-in, does not link it).
 * Conventions as rmr.h: int status (RMR_OK / RMR_E_*), message through rmr_group_last_error, calls
 * asynchronous until rmr_group_sync / rmr_group_read_frame / rmr_group_save_bmp.
 */
#ifndef RMR_GROUP_H
#define RMR_GROUP_H

#include <stddef.h>
#include <stdint.h>
#include "rmr.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rmr_group rmr_group;

/* A group over n distinct HIP devices (devices[0] holds the reduced frame): two rmr contexts and two
 * streams per device, one RCCL communicator per device (ncclCommInitAll). Graphics::Init for n GPUs. */
int  rmr_group_create(rmr_group** out, const int* devices, int n);
void rmr_group_destroy(rmr_group* g);
const char* rmr_group_last_error(const rmr_group* g);
int  rmr_group_size(const rmr_group* g);
/* Member m's context k (k = 0, 1: the two frame contexts), for settings the group does not forward
 * (rmr_set_jit, rmr_set_culling, ...); apply them to both contexts of every member. */
rmr_ctx* rmr_group_context(rmr_group* g, int member, int k);

/* Forwarded to every context of every member (rmr.h semantics; image size applied at reload). */
int rmr_group_set_image_size(rmr_group* g, int w, int h);
int rmr_group_set_params(rmr_group* g, const rmr_params* p);
int rmr_group_set_view(rmr_group* g, const float eye[3], const float ray00[3], const float ray01[3],
                       const float ray10[3], const float ray11[3]);
int rmr_group_load_scene_json(rmr_group* g, int variant, const char* json, size_t len);
int rmr_group_load_builtin_scene(rmr_group* g, int variant);
int rmr_group_set_env_map(rmr_group* g, const uint8_t* rgba8, int w, int h);
/* Graphics::Reload: apply the image size, allocate the members' frame buffers, partition the tiles
 * (tile_size: a positive multiple of 8; default 32). */
int rmr_group_set_tile_size(rmr_group* g, int tile_size);
int rmr_group_reload(rmr_group* g);

/* One frame: samples 0 .. nspp-1 of every pixel, sample k seeded with times[k] (the running mean of
 * RM1:600-612 from sample 0), each member its tiles, then the frame's reduce onto member 0.
 * Asynchronous; bitwise equal to rmr_render_spp of the whole image on one context. */
int rmr_group_render_frame(rmr_group* g, const float* times, uint32_t nspp);
int rmr_group_sync(rmr_group* g);
/* The last frame (after its reduce), RGBA32F, row 0 = top; synchronises. */
int rmr_group_read_frame(rmr_group* g, float* rgba, size_t bytes);
/* Graphics::SaveImage of the last frame (rmr_encode_bmp). */
int rmr_group_save_bmp(rmr_group* g, const char* path);
/* Member m's kernel statistics (its two contexts summed; trace_ms = summed trace-kernel time). */
int rmr_group_get_stats(rmr_group* g, int member, rmr_stats* out);
int rmr_group_reset_stats(rmr_group* g);

/* Host only (no GPU): the tiles (tx, ty) of member m of n for a w x h image, in the order that member
 * renders them; writes up to cap pairs into tiles_xy and returns the member's tile count (< 0: bad
 * arguments). The partition of raymarchrenderer_amd.multi_gpu.tile_partition. */
int rmr_group_partition(int w, int h, int tile_size, int member, int n, int32_t* tiles_xy, int cap);

#ifdef __cplusplus
}
#endif
#endif /* RMR_GROUP_H */
