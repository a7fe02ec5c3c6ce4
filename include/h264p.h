/*
 * h264p.h -- C ABI of the repo's own CPU entropy / syntax stage.
 *
 * The caller side of the reconstruction boundary (include/h264r.h): an Annex-B byte
 * stream is parsed on the host -- NAL units, SPS / PPS, slice headers, the CAVLC and
 * CABAC macroblock layer and residuals, motion-vector prediction (P_Skip, B direct spatial /
 * temporal), reference picture marking and list construction -- and every picture is
 * handed to the h264r ABI exactly as the reference parser + drop-in shim hand it
 * (shim/decoder_h264r.cc): h264r_picture_begin, h264r_mb_submit per MB, h264r_picture_end.
 * Decoded pictures come back in output order (POC order inside each IDR period).
 *
 *   reference (R/src/codec/h264/)                    here (arrow-h264_amd/parser/h264p.cc)
 *   ldecod.cc decode_one_frame, slice_data.cc:636-660  h264p_decode (NAL loop, picture boundary)
 *   interpret_rbsp.cc:625-777 slice_header              parse_slice_header
 *   interpret_rbsp.cc seq/pic_parameter_set_rbsp        parse_sps / parse_pps
 *   interpret_mb.cc:180-316 Macroblock::parse           SliceCtx::macroblock
 *   interpret_mv.cc:27-434 MV prediction, direct        SliceCtx::neighbour_mv / predict_mv / direct_*
 *   interpret_residual.cc:64-174 (CAVLC), 315-419        SliceCtx::block_cavlc / block_cabac / residual
 *     (CABAC), 421-494
 *   interpret.cc:308-432 cabac_engine_t                Cabac (dec / bypass / term, u / tu / ueg)
 *   interpret_se.cc, neighbour.cc:415-764 (CABAC ctx)   SliceCtx::cabac_* / cbf_inc
 *   slice_ref_list.cc:88-341, 885-964 ref lists         Decoder::init_lists / modify_list
 *   framebuf/dpb.cc marking (sliding window, MMCO)      Decoder::mark_picture
 *
 * The reconstruction calls are resolved at link time: against libh264r.so (MI355X) for the
 * product, against the CPU implementation of the same ABI in tests.  Status codes are the
 * h264r ones (H264R_OK / H264R_E*).  H264R_EUNSUPPORTED: MBAFF, FMO, data partitioning, formats
 * other than 4:2:0, 4:0:0 and 4:2:2 (frame pictures) or 4:4:4 (CAVLC, frame pictures, no separate
 * colour planes) 8-bit, POC type 1, MMCO 5, SI slices (as in the reconstruction path).
 */
#ifndef H264P_H_
#define H264P_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct h264p_dec h264p_dec;

/* One decoded picture in output order: planes of the coded size (16 W x 16 H luma,
 * pitch = width), the SPS cropping window in luma samples (frame_crop_*_offset x 2), its
 * POC and its IDR period (output order = (period, poc)). */
typedef struct h264p_frame {
    const uint8_t* y;
    const uint8_t* u;
    const uint8_t* v;
    int32_t width, height;
    int32_t crop_left, crop_right, crop_top, crop_bottom;
    int32_t poc;
    int32_t period;
    int32_t chroma_format;   /* chroma_format_idc: 1 (u, v: 8 W x 8 H), 2 (8 W x 16 H), 3 (16 W x 16 H) or
                                0 (4:0:0: no u, v) */
} h264p_frame;

/* Output callback: return 0 to continue, non-zero to stop decoding (h264p_decode then
 * returns that value). */
typedef int (*h264p_output_fn)(void* user, const h264p_frame* frame);

/* device: the GPU ordinal handed to h264r_create. */
int h264p_create(h264p_dec** out, int device);
int h264p_destroy(h264p_dec* dec);
/* Decode a complete Annex-B byte stream; every picture is output before it returns. */
int h264p_decode(h264p_dec* dec, const uint8_t* data, size_t size, h264p_output_fn out, void* user);
/* Text of the last error (which syntax element / which check), "" after success. */
const char* h264p_last_error(const h264p_dec* dec);

#ifdef __cplusplus
}
#endif
#endif /* H264P_H_ */
