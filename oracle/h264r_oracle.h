/*
 * h264r_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of luuvish/arrow-h264's macroblock-reconstruction path
 * (H/ = R/src/codec/h264/): decoder/decoder.cc, transform.cc,
 * intra_prediction.cc, inter_prediction.cc, deblock.cc, operating on the
 * canonical formats of include/h264r.h.  It is the checker for the HIP path
 * and the CPU baseline of bench.py; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  Nothing in the product links it.
 *
 * Parity pinning: outputs of the compiled reference itself (oracle/_ref,
 * built from /root/reference by oracle/Makefile) on the same seeded inputs,
 * committed as digests + crops under tests/golden/.
 */
#ifndef H264R_ORACLE_H_
#define H264R_ORACLE_H_

#include "h264r.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_picture {
    int                 width_mbs, height_mbs;
    const h264r_mb*     mbs;          /* [W*H]                                   */
    const int16_t*      levels;       /* pool, indexed by mb.coef_off            */
    const uint32_t*     mv;           /* [2][4H][4W]                             */
    const int8_t*       ref_idx;      /* [2][4H][4W]                             */
    const h264r_slice*  slices;
    const h264r_pic*    pic;
    const h264r_quant*  quant;
    const uint8_t*      ref_planes[H264R_MAX_SLOTS][3];   /* host planes per DPB slot */
    uint8_t*            out[3];       /* Y, Cb, Cr (unpadded, pitch = width)     */
    int                 chroma_format;/* 0 = 4:0:0 (luma only), 2 = 4:2:2 (chroma W/2 x H), 3 = 4:4:4 (planes of the
                                         luma size), else 4:2:0 */
} oracle_picture;

/* Transform::init/set_quant with flat matrices (transform.cc:173-180, 259-302). */
void oracle_quant_init_flat(h264r_quant* q);

/* Decoder::decode for every MB in raster order (slice_data.cc:636-661) followed by
 * Deblock::deblock (deblock.cc:622-656).  Returns 0 or a negative status. */
int  oracle_decode_picture(const oracle_picture* p);

/* Same, reconstruction only (no deblocking) -- used to localise mismatches. */
int  oracle_reconstruct_picture(const oracle_picture* p);
int  oracle_deblock_picture(const oracle_picture* p);

/* Decode n pictures on `threads` std::threads-equivalent pthreads (CPU baseline). */
int  oracle_decode_pictures(const oracle_picture* pics, int n, int threads);

#ifdef __cplusplus
}
#endif
#endif
