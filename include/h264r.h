/*
 * h264r.h -- C ABI of the MI355X-native H.264 macroblock-reconstruction path.
 *
 * This header is the drop-in boundary for the post-entropy hot path of
 * luuvish/arrow-h264 (`R/` = reference root, `H/` = R/src/codec/h264/):
 *
 *   reference interface                          replaced by (this header)
 *   -------------------------------------------  ------------------------------------------
 *   Decoder::assign_quant_params  decoder.cc:59   h264r_quant_init_flat / h264r_quant_init_lists
 *     (-> Transform::init/set_quant transform.cc:173-302)
 *   Decoder::coeff_luma_dc/ac,    decoder.cc:81-96 levels are written RAW (not dequantised) into
 *   Decoder::coeff_chroma_dc/ac                    the per-MB compacted level block described
 *   Decoder::transform_luma_dc,   decoder.cc:98-105 below (dequant + DC Hadamard move to the GPU)
 *   Decoder::transform_chroma_dc
 *   Decoder::decode(mb_t&)        decoder.cc:65-79 h264r_mb_submit   (one MB, host buffers) or
 *                                                   h264r_decode_batch (device-resident arrays)
 *   Decoder::deblock_filter       decoder.cc:107   h264r_picture_end  (recon + deblock + readback)
 *   storable_picture planes       picture.cc:17-83 h264r_set_ref / output planes (8-bit, unpadded)
 *
 * All entry points are extern "C", take plain pointers and sizes, and return
 * an int status (H264R_OK == 0, negative on error).  No exceptions cross the
 * boundary; the reference's void/assert/exit() error convention
 * (decoder.h:301-338, ldecod.cc:33-48) becomes status codes.
 *
 * Data formats (all little-endian, 4:2:0, 8-bit; frame pictures, field pictures (PAFF) and MBAFF
 * frames, h264r_pic.structure below):
 *   - h264r_mb       32-byte MB record (subset of mb_t, macroblock.h:78-135).
 *   - levels         int16 pool; each MB owns a compacted block at mb.coef_off
 *                    (in int16 units, multiple of 8):
 *                      for b8 in 0..3 with (cbp & 1<<b8): 64 levels
 *                          4x4 transform: 4 sub-blocks (raster inside the 8x8) x 16
 *                                         raster levels; 8x8 transform: 64 raster levels
 *                      if cbp_chroma == 2: 128 levels = Cb 4x16 then Cr 4x16
 *                                         (raster per 4x4 block, index 0 unused)
 *                      if I_16x16:        16 luma DC levels (raster of the 4x4 DC matrix)
 *                      if cbp_chroma != 0: 8 chroma DC levels (Cb c00 c01 c10 c11, Cr ...)
 *                      I_PCM:             384 raw samples as bytes (Y 256, Cb 64, Cr 64)
 *                    Levels are the entropy decoder's levels placed at their raster
 *                    position (inverse zig-zag done by the producer, transform.cc:307-386).
 *   - motion         per 4x4 block, per list: uint32 mv (int16 x in low half, int16 y
 *                    in high half, quarter-pel) and int8 ref_idx (-1 = list unused),
 *                    arrays [list][H4][W4] (pic_motion_params, picture.h:66-71).
 *   - planes         uint8 Y [H][W], Cb/Cr [H/2][W/2], pitch == width, no padding
 *                    (the reference pads by edge replication, picture.cc:182-205;
 *                     the GPU clamps coordinates instead -- equivalent).
 *
 * 4:4:4 (a context created with chroma_format_idc 3; frame pictures, 8-bit): every colour plane
 * is coded and reconstructed like luma (decode_one_component decoder.cc:65-79), so
 *   - planes         Cb / Cr are [H][W] like Y, in the output, the batch planes and the DPB slots;
 *   - levels         an MB's block is three luma-like blocks, Y then Cb then Cr, each: for b8 with
 *                    (cbp & 1<<b8) 64 levels as above, then, if I_16x16, its 16 DC levels;
 *                    cbp_chroma must be 0 (CodedBlockPatternChroma, 7.4.5); I_PCM: 768 raw
 *                    samples (Y, Cb, Cr 256 each), and 256 readable bytes after the MB's block;
 *   - h264r_mb       qp_c[] / qp_scaled[1..2] are the Cb / Cr QPs (deblocking / dequantisation),
 *                    cbp_blks the luma plane's non-zero mask (deblock.cc:135,212 read cbp_blks[0]);
 *                    chroma_mode is not used;
 *   - h264r_slice    wp_weight / wp_offset [..][..][1..2] with chroma_log2_wd weight Cb / Cr;
 *   - h264r_quant    scale4x4 / scale8x8 [..][1..2] are the Cb / Cr lists (8x8 lists 8..11).
 * The library decodes a 4:4:4 batch as three launch sequences of the 4:2:0 kernels, plane pl in
 * the luma slots.
 *
 * 4:2:2 (a context created with chroma_format_idc 2; frame pictures, 8-bit; not SP slices): Cb / Cr
 * carry 8 x 16 samples per MB, so
 *   - planes         Cb / Cr are [H][W/2] (half the luma width, the luma height), in the output, the
 *                    batch planes and the DPB slots;
 *   - levels         the luma part first, then chroma: for b8 with (cbp & 1<<b8) 64 levels as above;
 *                    if I_16x16, its 16 DC levels; if cbp_chroma == 2, 256 levels = Cb 8x16 then
 *                    Cr 8x16 (4x4 blocks in raster order of the 2 x 4 block grid, raster per block,
 *                    index 0 unused); if cbp_chroma != 0, 16 chroma DC levels (Cb then Cr, each the
 *                    raster of the 2-wide, 4-high DC matrix); I_PCM: 512 raw samples (Y 256, Cb 128,
 *                    Cr 128, raster);
 *   - deblocking     a transform-8x8 MB's chroma rows 4 and 12 take the bS of 8.7.2.1, which the
 *                    reference leaves unset.
 * The library decodes the luma by the 4:2:0 kernels and the chroma by its own kernels (DESIGN.md
 * section 4e).
 *
 * 4:0:0 (a context created with chroma_format_idc 0, monochrome; frame pictures, 8-bit; not SP
 * slices): there is no chroma (decoder.cc:199, picture.cc:34), so
 *   - planes         Y only: out_u / out_v of a batch and u / v of h264r_set_ref may be NULL and are
 *                    never written or read, nor u / v of h264r_picture_end / h264r_picture_wait;
 *   - levels         the luma part only: for b8 with (cbp & 1<<b8) 64 levels as above, then, if
 *                    I_16x16, its 16 DC levels; cbp_chroma must be 0; I_PCM: 256 raw samples, and
 *                    128 readable bytes after the MB's block;
 *   - h264r_mb       qp_c[] / qp_scaled[1..2] / chroma_mode are not used;
 *   - h264r_slice    the chroma weights are not used.
 * The library decodes the luma by the 4:2:0 kernels alone.  > 8-bit is
 * H264R_EUNSUPPORTED.
 */
#ifndef H264R_H_
#define H264R_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H264R_ABI_VERSION 4

/* ---- status codes ---------------------------------------------------------- */
#define H264R_OK               0
#define H264R_EINVAL          -1   /* bad argument / unsupported configuration   */
#define H264R_ENOMEM          -2   /* device or host allocation failed           */
#define H264R_EDEVICE         -3   /* HIP runtime error                          */
#define H264R_ESTATE          -4   /* call out of order (e.g. mb before begin)   */
#define H264R_EUNSUPPORTED    -5   /* valid H.264 but not on this path (MBAFF..) */
#define H264R_ENODEVICE       -6   /* no usable GPU / kernels not loaded         */

/* ---- limits ---------------------------------------------------------------- */
#define H264R_MAX_REFS        16   /* per list, frame pictures                   */
#define H264R_MAX_SLOTS       32   /* DPB slots addressable by ref tables        */
#define H264R_MAX_SLICES      256  /* per picture                                */

/* ---- mb_type values: identical to mb_t::mb_type (macroblock.h:48-76) -------- */
#define H264R_P_SKIP     0   /* also B_Skip / B_Direct_16x16 */
#define H264R_P_16x16    1
#define H264R_P_16x8     2
#define H264R_P_8x16     3
#define H264R_P_8x8      4
#define H264R_P_8x4      5
#define H264R_P_4x8      6
#define H264R_P_4x4      7
#define H264R_I_4x4      8
#define H264R_I_8x8      9
#define H264R_I_16x16   10
#define H264R_SI        11
#define H264R_I_PCM     12

/* ---- slice types (slice.h:29-35) ------------------------------------------- */
#define H264R_SLICE_P   0
#define H264R_SLICE_B   1
#define H264R_SLICE_I   2
#define H264R_SLICE_SP  3   /* inverse_transform_sp (transform.cc:1267-1300); QsC < 6 only: the reference
                               indexes LevelScale2[QsC] unreduced (:1230,1235), undefined beyond */
#define H264R_SLICE_SI  4   /* SI MBs (mb_type H264R_SI): EUNSUPPORTED -- the reference sends them through
                               mb_pred_inter with an out-of-range BLOCK_STEP row (decoder.cc:141-146,212-225) */

/* ---- h264r_mb.flags ---------------------------------------------------------- */
#define H264R_MBF_INTRA   0x01   /* mb_t::is_intra_block            */
#define H264R_MBF_T8x8    0x02   /* mb_t::transform_size_8x8_flag   */
#define H264R_MBF_BYPASS  0x04   /* mb_t::TransformBypassModeFlag (lossless: levels are the residual,
                                    DPCM by the block's ipred mode -- for inter MBs too, as the
                                    reference reads Intra4x4/8x8PredMode there, transform.cc:993,1008;
                                    an inter MB's chroma_mode must be 0, the parser's value) */
#define H264R_MBF_FIELD   0x08   /* mb_t::mb_field_decoding_flag (H264R_MBAFF_FRAME pictures only; both
                                    MBs of a pair carry the same value) */

/* 32-byte macroblock record (fields named after mb_t, macroblock.h:78-135). */
typedef struct h264r_mb {
    uint8_t  mb_type;        /* mb_t::mb_type                                        */
    uint8_t  flags;          /* H264R_MBF_*                                          */
    uint8_t  cbp;            /* CodedBlockPatternLuma | CodedBlockPatternChroma << 4 */
    int8_t   qp_y;           /* QpY   (deblock, deblock.cc:469-470)                  */
    int8_t   qp_c[2];        /* QpC[] (deblock)                                      */
    uint8_t  i16_mode;       /* Intra16x16PredMode                                   */
    uint8_t  chroma_mode;    /* intra_chroma_pred_mode                               */
    uint16_t cbp_blks;       /* cbp_blks[0] (non-zero 4x4 mask, deblock bS=2)        */
    uint16_t slice;          /* index into the picture's slice table (slice_nr)      */
    uint8_t  qp_scaled[3];   /* qp_scaled[] (dequant, transform.cc:400-401)          */
    uint8_t  pad0;
    uint32_t coef_off;       /* offset of the compacted level block, int16 units     */
    uint8_t  ipred[8];       /* Intra4x4PredMode[16] as nibbles (blkIdx order, low
                                nibble first) or Intra8x8PredMode[4] in nibbles 0..3 */
    uint8_t  pad1[4];
} h264r_mb;

/* Per-slice parameters (subset of slice_header_t + ref lists, slice.h:37-131). */
typedef struct h264r_slice {
    uint8_t  slice_type;           /* H264R_SLICE_*                                      */
    uint8_t  deblock_idc;          /* disable_deblocking_filter_idc                      */
    int8_t   filter_offset_a;      /* FilterOffsetA                                      */
    int8_t   filter_offset_b;      /* FilterOffsetB                                      */
    uint8_t  wp_mode;              /* 0 default, 1 explicit, 2 implicit (inter_prediction.cc:62-63,99-139) */
    uint8_t  luma_log2_wd;         /* luma_log2_weight_denom (5 when not explicit, interpret_rbsp.cc:722) */
    uint8_t  chroma_log2_wd;       /* chroma_log2_weight_denom                           */
    uint8_t  num_ref[2];
    uint8_t  qs_y;                 /* SP slices: QsY (slice_qs_delta, interpret_rbsp.cc:740-748)           */
    uint8_t  sp_switch;            /* SP slices: sp_for_switch_flag                                        */
    int8_t   qs_c[2];              /* SP slices: QsC[] of the slice's MBs (interpret_mb.cc:799-801)       */
    uint8_t  pad[3];
    int8_t   ref_slot[2][H264R_MAX_REFS];       /* RefPicList[l][i] -> DPB slot       */
    int8_t   wp_weight[2][H264R_MAX_REFS][3];   /* pred_weight_l[l][pl][i].weight     */
    int8_t   wp_offset[2][H264R_MAX_REFS][3];   /* pred_weight_l[l][pl][i].offset     */
    int16_t  implicit_w1[H264R_MAX_REFS][H264R_MAX_REFS]; /* weight1 for (ref0,ref1), w0 = 64-w1 */
} h264r_slice;

/* Dequantisation tables (Transform::InvLevelScale*, transform.cc:264-301). */
typedef struct h264r_quant {
    int16_t scale4x4[2][3][6][16];   /* [0 intra / 1 inter][plane][qp%6][raster] */
    int16_t scale8x8[2][3][6][64];
} h264r_quant;

/* Per-picture parameters. */
#define H264R_FRAME         0   /* PictureStructure FRAME (defines.h)                          */
#define H264R_TOP_FIELD     1   /* a field picture (field_pic_flag, slice_header bottom_field_flag */
#define H264R_BOTTOM_FIELD  2   /* 0 / 1; interpret_rbsp.cc): height_mbs is the FIELD's height  */
/* Field pictures (ABI 3).  A field picture is reconstructed and deblocked as a picture of
 * PicHeightInMbs = FrameHeightInMbs / 2 rows (slice_header: PicHeightInMbs; the reference
 * decodes it into a field storable_picture, picture.cc:17-83, and deblocks it on its own,
 * exit_picture picture.cc:253), with three differences the kernels apply:
 *   - its references are FIELDS of the DPB's frames: RefPicList entry = slot | H264R_REF_BOTTOM
 *     for the bottom field of DPB slot `slot`, the plain slot for its top field; the plane is
 *     read as every second row of the slot's frame (dpb_split_field picture.cc:408-470 without
 *     the copy), clamped to the field's rows;
 *   - chroma MC of a reference field of the other parity moves by -2 (top field predicting from
 *     a bottom field) / +2 (bottom from top) quarter luma rows (get_block_chroma
 *     inter_prediction.cc:352-355);
 *   - bS: |dmv_y| >= 2 instead of 4 (mvlimit, deblock.cc:86,164), and intra / SP MB edges that
 *     are horizontal get bS 3, not 4 (cond_bS4, deblock.cc:103-107,184-189).
 * Reference identity (deblocking) is (slot, parity).  DPB slots always hold frames: the
 * streaming API stores a field picture kept as a reference into its parity's rows of the slot
 * (dpb_combine_field_yuv picture.cc:578-622 without the copy), so the two fields of a frame
 * share one slot and a frame picture may later reference the frame they make up. */
#define H264R_REF_BOTTOM  0x40
/* MBAFF frames (ABI 4, mb_adaptive_frame_field_flag: MbaffFrameFlag of slice_header, macroblock
 * pairs that are each coded as two frame MBs or as two field MBs, H264R_MBF_FIELD).  A frame picture
 * of the context's size whose MBs are stored as the reference stores them (mb_t::mb, the position
 * slice_data.cc gives an MB of address a: x = (a / 2) % W, y = 2 ((a / 2) / W) + a % 2):
 *   - records  the record of MB address a is mbs[y * W + x] (pair row r: its top MB in row 2r, its
 *              bottom MB in row 2r + 1), and the streaming API's mb_addr is that index, y * W + x;
 *   - motion   rows 4 y .. 4 y + 3 of the [H4][W4] arrays hold MB (x, y)'s blocks (the reference's
 *              mv_info rows, inter_prediction.cc:456), in its own frame or field rows;
 *   - ref_idx  a field MB's refIdx counts fields (0 .. 2 num_ref - 1): field refIdx / 2 of the slice's
 *              frame list, the same parity as the MB when refIdx is even (get_ref_pic dpb.cc:1046-1055);
 *              its explicit weights are those of refIdx / 2 (inter_prediction.cc:66,100-101);
 *   - output   the frame: a field MB's rows are every second row of its pair, from the pair's
 *              first (top MB) or second row (bottom MB) -- the picture after MbAffPostProc
 *              (deblock.cc:581-620), which the reference applies before the loop filter.
 * Intra prediction takes its neighbours where Neighbour::get_neighbour finds them (neighbour.cc:
 * 123-173: the geometric sample of the frame, the MB holding it), and the loop filter follows
 * Deblock::strength / filter_edge (deblock.cc:78-289, 418-535): mixed frame / field edges, the
 * top edge of a frame MB under a field pair filtered as two field edges, mvlimit 2 in field MBs.
 * 4:2:0 only; not with SP slices, lossless MBs or implicit weights (H264R_EUNSUPPORTED). */
#define H264R_MBAFF_FRAME   3
typedef struct h264r_pic {
    int32_t  constrained_intra_pred;  /* pps.constrained_intra_pred_flag */
    int32_t  num_slices;
    int32_t  poc;                     /* informational (implicit weights are precomputed) */
    int32_t  structure;               /* H264R_FRAME / H264R_TOP_FIELD / H264R_BOTTOM_FIELD / H264R_MBAFF_FRAME */
} h264r_pic;

/* A batch of same-sized pictures whose arrays are already resident on the device.
 * Per-picture strides: MBs W*H records; motion 2*(4H)*(4W) entries; slices
 * `slice_stride` entries; planes (16W)*(16H) bytes (Y) and (8W)*(8H) (Cb, Cr).
 * `ref_planes` is a device array of 3*H264R_MAX_SLOTS device pointers
 * (Y,Cb,Cr per DPB slot) to full-size planes (frames: 2 * height_mbs MB rows when the
 * batch's pictures are fields, H264R_TOP_FIELD above); MC reads whole dwords, so each
 * plane must be followed by H264R_PLANE_SLACK readable bytes (the slots of
 * h264r_set_ref / h264r_ref_planes are).  `ref_planes_stride` (ABI 2): 0 = that one
 * table serves every picture of the batch; otherwise picture p reads its own table at
 * ref_planes + p * ref_planes_stride (>= 3*H264R_MAX_SLOTS pointers apart) -- a batch of
 * pictures from different streams, each with its own DPB (the reference keeps one DPB per
 * decoder, dpb.cc:1046-1054 get_ref_pic; bench.py's dependent chains). */
#define H264R_PLANE_SLACK 64
typedef struct h264r_batch {
    int32_t             num_pics;
    int32_t             width_mbs;
    int32_t             height_mbs;
    int32_t             slice_stride;
    const h264r_mb*     mbs;
    const int16_t*      levels;
    const uint32_t*     mv;
    const int8_t*       ref_idx;
    const h264r_slice*  slices;
    const h264r_pic*    pics;
    const h264r_quant*  quant;       /* one table per picture */
    const uint8_t* const* ref_planes;
    uint8_t*            out_y;
    uint8_t*            out_u;       /* NULL allowed on a 4:0:0 context */
    uint8_t*            out_v;
    int64_t             ref_planes_stride;   /* pointers; 0 = one table for the batch (above) */
    int32_t             mbaff;       /* ABI 4: nonzero = every picture is an H264R_MBAFF_FRAME (its own
                                        launch sequence, whole pictures only); 0 = frames / fields */
    int32_t             colour_plane;/* ABI 4, separate_colour_plane_flag (JV) on a 4:4:4 context: 0 = off;
                                        k + 1 = every picture is colour plane k (colour_plane_id) of its
                                        frame: 4:0:0 records and levels (a PCM MB's block followed by 128
                                        readable bytes), reconstructed and deblocked as luma with plane k's
                                        scaling lists (transform.cc:402) from plane k of the DPB slots
                                        (inter_prediction.cc:175-177) into out_y / out_u / out_v for
                                        k = 0 / 1 / 2 (make_frame_picture_JV deblock.cc:555-579); the other
                                        two output planes are not written.  The reference scales an
                                        Intra_16x16 DC of plane k by the Y intra list (transform.cc:831-
                                        836); the library by plane k's -- the same unless the first
                                        entries of the two intra 4x4 lists differ */
} h264r_batch;

typedef struct h264r_ctx h264r_ctx;

/* ---- library / device ---------------------------------------------------------- */
int  h264r_abi_version(void);
/* Human-readable text for a status code. */
const char* h264r_strerror(int status);
/* Number of usable gfx950 devices (0 when no GPU; never falls back to the CPU). */
int  h264r_device_count(void);

/* ---- quantisation tables (Transform::init + set_quant, transform.cc:173-302) -- */
/* Flat_4x4_16 / Flat_8x8_16 matrices (no scaling lists). */
int  h264r_quant_init_flat(h264r_quant* q);
/* qmatrix[12] already resolved by the caller (fall-back rules A/B, transform.cc:178-254):
 * lists 0..5 are 16-entry 4x4 lists (Intra Y,Cb,Cr, Inter Y,Cb,Cr), 6..11 64-entry
 * 8x8 lists (Intra Y, Inter Y, Intra Cb, Inter Cb, Intra Cr, Inter Cr), raster order. */
int  h264r_quant_init_lists(h264r_quant* q, const int32_t* const qmatrix[12]);

/* ---- context ------------------------------------------------------------------- */
/* chroma_format_idc 0 (4:0:0), 1 (4:2:0), 2 (4:2:2) or 3 (4:4:4, above) and bit_depth 8 (other
 * formats: H264R_EUNSUPPORTED). */
int  h264r_create(h264r_ctx** out, int device, int max_width_mbs, int max_height_mbs,
                  int chroma_format_idc, int bit_depth);
int  h264r_destroy(h264r_ctx* ctx);

/* Load (host -> device) a decoded reference picture into DPB slot `slot`
 * (storable_picture planes after deblock, exit_picture picture.cc:239-269). */
int  h264r_set_ref(h264r_ctx* ctx, int slot, const uint8_t* y, const uint8_t* u,
                   const uint8_t* v, int width_mbs, int height_mbs);

/* ---- per-picture streaming API (the Decoder shim drives this) ---------------------- */
/* height_mbs: the picture's own height (a field picture: FrameHeightInMbs / 2, pic->structure
 * naming its parity); DPB slots it reads or keeps into are frames of the context's size. */
int  h264r_picture_begin(h264r_ctx* ctx, int width_mbs, int height_mbs,
                         const h264r_pic* pic, const h264r_slice* slices,
                         const h264r_quant* quant);
/* Decoder::decode(mb) for MB address mb_addr.  `levels` is this MB's compacted
 * level block (n_levels int16), mv/ref_idx are its 16 4x4 entries per list in
 * raster order ([list][16]). */
int  h264r_mb_submit(h264r_ctx* ctx, int mb_addr, const h264r_mb* mb,
                     const int16_t* levels, int n_levels,
                     const uint32_t* mv /*[2][16]*/, const int8_t* ref_idx /*[2][16]*/);
/* Decoder::deblock_filter: reconstruct + deblock on the GPU, copy planes back.
 * If keep_as_ref_slot >= 0 the result also stays on the device as that DPB slot.
 * (H264R_ESTATE while a picture of the asynchronous form below is outstanding.) */
int  h264r_picture_end(h264r_ctx* ctx, uint8_t* y, uint8_t* u, uint8_t* v,
                       int keep_as_ref_slot);
/* The same, split so that the host parses the next picture while the GPU reconstructs this
 * one: h264r_picture_end_async enqueues the upload, the reconstruction, the DPB-slot copy and
 * the readback into pinned staging on the context's stream and returns; the next
 * h264r_picture_begin may follow at once (two pictures are staged; a third begin before a
 * wait is H264R_ESTATE).  A later picture may reference keep_as_ref_slot right away (stream
 * order).  h264r_picture_wait blocks until the OLDEST outstanding picture is done and copies
 * its planes out (NULL skips a plane); it reports that picture's device-side failures
 * (H264R_EDEVICE), as h264r_check does for the synchronous form. */
int  h264r_picture_end_async(h264r_ctx* ctx, int keep_as_ref_slot);
int  h264r_picture_wait(h264r_ctx* ctx, uint8_t* y, uint8_t* u, uint8_t* v);

/* ---- batch API (bench / throughput mode): arrays already on the device ---------- */
/* Launches recon + deblock for every picture of the batch on `stream`
 * (a hipStream_t, NULL = the context's stream, a blocking stream: ordered with the
 * legacy NULL stream).  Asynchronous.
 * Threading / residency contract: a context is driven by one host thread; its scratch
 * is reused by every launch, so a launch on a different stream than the previous one
 * first waits for the previous one (an event, inserted by the library).  The intra
 * kernel k_intra_levels is persistent and separates dependency levels with a grid
 * barrier sized from the occupancy query: kernels of OTHER contexts or libraries
 * running concurrently on the same device may delay it (every wait is bounded; an
 * expired wait is reported by h264r_check as H264R_EDEVICE, never silently).  It is
 * launched plainly (H264R_COOP=1: a cooperative launch, whose runtime check refuses a grid
 * that cannot be resident).  Launches deblocked by the split walk also use the context's
 * side stream (joined back to the launch stream by an event before the call returns). */
int  h264r_decode_batch(h264r_ctx* ctx, const h264r_batch* batch, void* stream);

/* Slice-sharded form of h264r_decode_batch (multi-GPU): reconstruct and
 * deblock only MB rows [row0, row1) of every picture of the batch.  The band must start
 * at a slice boundary and must not be deblocked across its top edge (its first slice has
 * disable_deblocking_filter_idc 1, or 2 with a slice edge there; deblock.cc:247-253);
 * slices never predict across each other (intra_prediction.cc:145-152), so the band is
 * then independent of the rows outside it.  Motion compensation still reads whole
 * reference pictures.  A band whose top edge would be filtered is reported by
 * h264r_check() as H264R_EDEVICE.  Replaces nothing in the reference (its decoder is
 * single-threaded); the slice walk it parallelises is slice_data.cc:640-650. */
int  h264r_decode_batch_rows(h264r_ctx* ctx, const h264r_batch* batch, int row0, int row1, void* stream);
/* Device pointer of DPB slot planes (for building h264r_batch.ref_planes). */
int  h264r_ref_planes(h264r_ctx* ctx, int slot, uint8_t** y, uint8_t** u, uint8_t** v);

/* ---- instrumentation ------------------------------------------------------------- */
/* Average device time (ms) per h264r_decode_batch of the launches made since timing was
 * enabled, measured with HIP events on each launch's stream: out[0] the deblocking records
 * and the inter / I_PCM reconstruction (k_inter4r + k_inter_sp), out[1] the intra
 * kernels (k_level + k_level_scatter + k_intra_levels + k_intra_pic), out[2]
 * deblocking (k_deblock2, or the split walk k_deblock2y + k_deblock2c), out[3] the whole batch (the wall time of the launch
 * sequence on the launch stream; under the overlapped schedule out[0..2] are busy times that
 * overlap).  Returns H264R_OK or an error. */
int  h264r_last_timing(h264r_ctx* ctx, float out_ms[4]);
int  h264r_set_timing(h264r_ctx* ctx, int enable);
/* Debug hook: H264R_DBG_NO_DEBLOCK skips the loop filter (reconstruction only, to
 * localise a mismatch against the oracle's pre-deblock planes). */
#define H264R_DBG_NO_DEBLOCK 1
/* H264R_DBG_INTRA_WALK reconstructs every intra MB with the wavefront walk instead of
 * the dependency-level schedule (both are bit-exact; this exercises the walk alone). */
#define H264R_DBG_INTRA_WALK 2
/* The loop filter has three schedules (all bit-exact): k_deblock2 walks bands of 4 MB rows of
 * 2 pictures per wave, 8 lanes per (picture, row) (launches of >= H264R_DB2S_MAX x 68
 * picture-MB-rows, 512 1080p pictures by default); below that the split walk runs the luma
 * and the chroma planes' band walks as separate waves (H264R_DBG_DEBLOCK_SPLIT); k_deblock
 * spreads one MB over 32 lanes (with H264R_DB2S_MAX=0, launches below H264R_DEBLOCK2_MIN x 68
 * picture-MB-rows).  These flags force one of them. */
#define H264R_DBG_DEBLOCK_MB   4
#define H264R_DBG_DEBLOCK_ROWS 8
/* Both schedules keep a picture's (k_deblock) or a 2-picture group's (k_deblock2) rows on
 * one XCD and hand records over in that XCD's L2; H264R_DBG_DEBLOCK_GLOBAL uses one
 * ticket counter and write-through records instead (any wave on any XCD). */
#define H264R_DBG_DEBLOCK_GLOBAL 16
/* Test hook for the bounded waits: every intra MB goes through the wavefront walk, whose
 * row-to-row waits then ask for progress that never comes, under a 10 ms bound.  The
 * launch drains and h264r_check returns H264R_EDEVICE (the output is invalid).  The
 * bound of every wait is wall time: 2 s by default (environment H264R_WAIT_MS). */
#define H264R_DBG_WAIT_TEST 32
/* The overlapped schedule (off by default: measured slower): large batches
 * cut into 4 picture chunks (H264R_OVERLAP=<n> sets the count), chunk k deblocked on the
 * context's side stream while chunk k + 1 is reconstructed on the launch stream. */
#define H264R_DBG_OVERLAP 64
/* H264R_DBG_DEBLOCK_SPLIT forces the split band walk: the luma planes' walk (k_deblock2y) and the
   chroma planes' (k_deblock2c) as separate waves running together -- the planes filter
   independently, and each walk's step is shorter than the combined one. */
#define H264R_DBG_DEBLOCK_SPLIT 128
int  h264r_set_debug(h264r_ctx* ctx, int flags);
/* Wait for the context's work and report a device-side failure (a wavefront wait
 * that timed out): H264R_OK or H264R_EDEVICE. */
int  h264r_check(h264r_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* H264R_H_ */
