/*
 * h264r_synth.h -- seeded synthetic post-entropy workload generator.
 *
 * Produces canonical h264r inputs (include/h264r.h) with the distributions of
 * MB-type mixes per picture kind, QP, CBP, level
 * statistics, quarter-pel motion over all 16 phases, intra modes drawn only
 * from the modes valid for the actual neighbour availability (the reference
 * asserts otherwise, intra_prediction.cc:191-873).  Deterministic: the same
 * (cfg, picture index) always yields the same bytes on every host.  Used by the
 * benchmark (GPU inputs + CPU baseline), the parity tests and the reference
 * fixture driver -- identical inputs everywhere.
 */
#ifndef H264R_SYNTH_H_
#define H264R_SYNTH_H_

#include "h264r.h"

#ifdef __cplusplus
extern "C" {
#endif

#define H264R_SYNTH_INTRA 0   /* config 2: all-intra                     */
#define H264R_SYNTH_P     1   /* config 3: P pictures (IPPP Main)         */
#define H264R_SYNTH_B     2   /* config 4/5: B pictures (IBBP High)       */

/* Upper bound of int16 level-pool entries one MB can use: 4:2:0 4*64+128+16+8 (rounded to 8);
 * 4:2:2 4*64+16+256+16; 4:4:4 three luma-like blocks 3*(4*64+16), and a PCM MB's plane-2 view
 * reads 128 entries past its 384 (include/h264r.h, 4:4:4). */
#define H264R_SYNTH_CHROMA_400 4       /* h264r_synth_cfg.chroma_format for 4:0:0 (0 stays 4:2:0) */

#define H264R_SYNTH_MAX_LEVELS_PER_MB 416
#define H264R_SYNTH_MAX_LEVELS_PER_MB_422 544
#define H264R_SYNTH_MAX_LEVELS_PER_MB_444 816

typedef struct h264r_synth_cfg {
    int32_t  width_mbs, height_mbs;
    int32_t  kind;               /* H264R_SYNTH_*                                         */
    int32_t  num_slices;         /* contiguous MB-row bands                               */
    int32_t  deblock_idc;        /* disable_deblocking_filter_idc for every slice         */
    int32_t  filter_offset_a;    /* FilterOffsetA (even, -12..12)                         */
    int32_t  filter_offset_b;
    int32_t  transform8x8;       /* allow 8x8 transform / I_8x8 (High profile)            */
    int32_t  wp_mode;            /* P: 0/1, B: 0/1/2                                       */
    int32_t  constrained_intra;  /* pps.constrained_intra_pred_flag                       */
    int32_t  num_refs;           /* reference pictures (DPB slots 0..num_refs-1), <= 16   */
    int32_t  qp_min, qp_max;
    int32_t  pcm_permille;       /* I_PCM MBs per 1000 MBs (0 for the bench configs)      */
    int32_t  intra_permille;     /* intra MBs in P/B pictures (default 100)               */
    int32_t  mv_range_x, mv_range_y;   /* integer-pel MV range (default 64 / 32)          */
    int32_t  lossless_permille;  /* sps.qpprime_y_zero_transform_bypass_flag when > 0: this
                                    many MBs per 1000 get QP'Y 0, and every MB at QP'Y 0 is a
                                    TransformBypassModeFlag MB (interpret_mb.cc:804); inter
                                    bypass MBs carry random Intra4x4/8x8PredMode values, which
                                    the reference's bypass DPCM reads for them (transform.cc:993,1008) */
    int32_t  sp_slices;          /* P pictures: every slice an SP slice (QsY 0..5 -- the reference's
                                    itrans_sp_cr indexes LevelScale2 by QsC unreduced, transform.cc:1230,
                                    so only QsC < 6 has defined results -- sp_for_switch_flag random)   */
    int32_t  structure;          /* H264R_FRAME, or a field picture (H264R_TOP_FIELD / H264R_BOTTOM_FIELD):
                                    height_mbs is then the field's height, num_refs counts reference
                                    FIELDS (list entries), taken from DPB frames 0 .. (num_refs+1)/2 - 1
                                    of 2 * height_mbs MB rows: the fields of frame slot s have POC
                                    4 s (top) and 4 s + 1 (bottom), the lists order them by POC as
                                    8.2.4.2.4/8.2.4.2.5 would (alternating parity); or H264R_MBAFF_FRAME:
                                    a frame of MB pairs (height_mbs even), each pair frame or field
                                    (H264R_MBF_FIELD) at random, slices of whole pair rows, a field MB's
                                    refIdx over the 2 num_refs fields (4:2:0; wp_mode 0/1; no SP,
                                    no lossless) */
    int32_t  chroma_format;      /* chroma_format_idc: 3 = 4:4:4 (every plane coded like luma: three
                                    luma-like level blocks per MB, CodedBlockPatternChroma 0, a PCM MB
                                    3 x 256 samples; frame pictures); 2 = 4:2:2 (chroma 8 x 16 per MB:
                                    8 chroma 4x4 blocks and 8 DC levels per plane, the layout of
                                    include/h264r.h; frame pictures); H264R_SYNTH_CHROMA_400 = 4:0:0 (luma
                                    only: cbp_chroma 0, a PCM MB 256 samples; frame pictures); anything
                                    else (0 -- the default -- or 1) = 4:2:0                              */
    uint64_t seed;
} h264r_synth_cfg;

/* Fill cfg with the defaults of a SURVEY config (2 intra, 3 P, 4/5 B) at the given size. */
int  h264r_synth_default(h264r_synth_cfg* cfg, int config_idx, int width_mbs, int height_mbs);

/* Generate picture `index` of the stream.  Caller-owned outputs:
 *   mbs[W*H], levels[W*H*H264R_SYNTH_MAX_LEVELS_PER_MB] (int16), mv[2*16*W*H],
 *   ref_idx[2*16*W*H], slices[cfg->num_slices], pic[1].
 * *n_levels receives the number of pool entries used. */
int  h264r_synth_picture(const h264r_synth_cfg* cfg, int index, h264r_mb* mbs, int16_t* levels,
                         int64_t* n_levels, uint32_t* mv, int8_t* ref_idx, h264r_slice* slices,
                         h264r_pic* pic);

/* Deterministic reference-picture content for DPB slot `slot` (smooth texture + noise). */
int  h264r_synth_refpic(uint64_t seed, int slot, int width_mbs, int height_mbs,
                        uint8_t* y, uint8_t* u, uint8_t* v);
/* The same for a chroma format (h264r_synth_cfg.chroma_format): 3 = 4:4:4, chroma planes of the
 * luma plane's size; 2 = 4:2:2, chroma planes of half the luma width and its full height;
 * H264R_SYNTH_CHROMA_400, the luma plane only (u, v may be NULL) (the 4:2:0 content of
 * h264r_synth_refpic otherwise). */
int  h264r_synth_refpic_fmt(uint64_t seed, int slot, int width_mbs, int height_mbs, int chroma_format,
                            uint8_t* y, uint8_t* u, uint8_t* v);

/* POC assigned to DPB slot `slot` (its frame; fields: + 0 top, + 1 bottom) / to the current
 * picture (a field's own POC) by the generator, and the number of DPB frames it references. */
int  h264r_synth_slot_poc(int slot);
int  h264r_synth_cur_poc(const h264r_synth_cfg* cfg);
int  h264r_synth_ref_frames(const h264r_synth_cfg* cfg);

/* Algorithmic bytes of a batch: R and W summed over the MBs. */
int  h264r_synth_algo_bytes(const h264r_mb* mbs, const int8_t* ref_idx, int width_mbs,
                            int height_mbs, int64_t* read_bytes, int64_t* write_bytes);

#ifdef __cplusplus
}
#endif
#endif
