/* h264r_group.h -- the multi-GPU exchange of slice bands behind the C ABI.
 *
 * One process per GPU.  When a picture shards into slice bands (slices never predict across
 * each other, intra_prediction.cc:145-152 / interpret_mv.cc:35-38, and deblocking idc 2 stops at
 * slice edges, deblock.cc:247-253), each rank reconstructs and deblocks its band of MB rows with
 * h264r_decode_batch_rows (h264r.h).  Every rank then needs, as a motion-compensation reference
 * of its next pictures, the rows of the other bands that its vectors can reach: this API moves
 * them.  The reference decoder is single-threaded (its slice walk is slice_data.cc:640-650), so
 * nothing in it is replaced; the interface is the library's own, and h264r/dist.py's
 * BandExchange is a thin caller of it.
 *
 * Transport: RCCL point-to-point (ncclSend / ncclRecv in one ncclGroupStart/End, over xGMI),
 * loaded from librccl at h264r_group_create -- the library does not link it, so a process that
 * never makes a group does not need it -- or the caller's own callbacks (h264r_transport; the
 * CPU rehearsal passes torch.distributed gloo operations).  Planes are device memory (device >= 0)
 * or, with a callback transport only, host memory (device < 0: the exchange packs with memcpy
 * and never touches a GPU).
 *
 * Layout: plane k of picture i starts at base[k] + i * stride[k] bytes (the h264r_batch out
 * planes: stride 256 * W * H for luma, 64 * W * H for chroma); rows are full width.  A peer's
 * segment of the staging buffers holds, per picture, its luma rows then its Cb then its Cr rows.
 */
#ifndef H264R_GROUP_H_
#define H264R_GROUP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H264R_GROUP_ID_BYTES   128   /* ncclUniqueId */
#define H264R_GROUP_MAX_RANKS  64
/* exchange modes */
#define H264R_XCHG_HALO        0     /* the rows within halo_mb_rows of the receiver's band      */
#define H264R_XCHG_ALLGATHER   1     /* every other band whole                                   */

typedef struct h264r_group h264r_group;

/* Caller-provided transport.  For one exchange the library calls start, then send / recv for
 * every peer it exchanges with (sends first, peers in increasing rank order), then finish,
 * which must return once every posted transfer has completed.  Buffers are host memory (device
 * planes are staged through pinned host buffers) and stay valid until finish returns.  Every
 * callback returns 0 on success; anything else fails the exchange with H264R_EDEVICE. */
typedef struct h264r_transport {
    void* user;
    int (*start)(void* user);
    int (*send)(void* user, int peer, const void* buf, size_t bytes);
    int (*recv)(void* user, int peer, void* buf, size_t bytes);
    int (*finish)(void* user);
} h264r_transport;

/* ncclGetUniqueId: made by one rank and handed to every other rank by the caller (any side
 * channel: a torch.distributed broadcast, MPI, a file).  H264R_ENODEVICE without librccl. */
int h264r_group_unique_id(uint8_t id[H264R_GROUP_ID_BYTES]);
/* An RCCL group of nranks processes (ncclCommInitRank: blocks until every rank has joined). */
int h264r_group_create(h264r_group** out, int device, int nranks, int rank,
                       const uint8_t id[H264R_GROUP_ID_BYTES]);
/* A group over the caller's transport (copied; `user` must outlive the group). */
int h264r_group_create_transport(h264r_group** out, int device, int nranks, int rank,
                                 const h264r_transport* transport);
int h264r_group_destroy(h264r_group* g);

/* The exchange plan, a pure function (no group, no device): bands[2 r], bands[2 r + 1] are rank
 * r's MB rows [row0, row1) (row1 <= row0: an empty band).  For every peer r, need[2 r .. 2 r + 1]
 * are the rows this rank receives from r and give[...] the rows it sends to r (row1 == row0 == 0:
 * none).  Halo mode: a rank with a band receives the rows of other bands within halo_mb_rows of
 * it; allgather mode: every rank receives every other band whole. */
int h264r_group_plan(int nranks, int rank, const int32_t* bands, int mode, int halo_mb_rows,
                     int32_t* need, int32_t* give);

/* Fix the picture size, the band plan and the capacity (pictures per exchange) of the group;
 * allocates its staging buffers.  May be called again (a new plan). */
int h264r_group_set_bands(h264r_group* g, int width_mbs, int height_mbs, const int32_t* bands,
                          int mode, int halo_mb_rows, int max_pics);

/* After this rank has decoded its band of num_pics pictures into the planes, bring in the rows
 * of the other bands the plan names, in place.  RCCL: enqueued on `stream` (a hipStream_t,
 * NULL = the legacy stream) and asynchronous, like h264r_decode_batch -- a decode of the next
 * pictures on the same stream reads the received rows.  Callback transport: returns when the
 * rows are in place.  A group's staging buffers are reused by every exchange: drive a group from
 * one stream (or order the streams), as a context. */
int h264r_group_exchange(h264r_group* g, int num_pics, uint8_t* y, uint8_t* u, uint8_t* v,
                         int64_t stride_y, int64_t stride_c, void* stream);

/* Bytes this rank sent / received over all exchanges so far, and the transfers it posted. */
int h264r_group_stats(h264r_group* g, int64_t* sent, int64_t* received, int64_t* transfers);

#ifdef __cplusplus
}
#endif
#endif /* H264R_GROUP_H_ */
