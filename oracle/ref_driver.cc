/*
 * ref_driver.cc -- TEST INFRASTRUCTURE ONLY.  Drives the *unmodified* reference
 * decoder (luuvish/arrow-h264, compiled from /root/reference by oracle/Makefile)
 * on one synthetic picture and writes its output planes, so that the oracle
 * restatement and the GPU path can be pinned to the reference's own bytes.
 *
 * It contains no reference code: it includes the reference headers and calls
 * the reference's per-MB boundary exactly as the parser would:
 *   Decoder::assign_quant_params  (slice_header.cc:185)
 *   Decoder::init                 (slice_data.cc:618)
 *   Decoder::coeff_luma_dc/ac, coeff_chroma_dc/ac, transform_luma_dc/chroma_dc
 *                                  (interpret_residual.cc:159-170, 405-415, 430, 475)
 *   Decoder::decode(mb)            (slice_data.cc:646), MBs in raster order
 *   Decoder::deblock_filter        (picture.cc:253)
 * Reference pictures are padded with the reference's own pad_buf (picture.cc:182).
 *
 * usage: ref_driver W H kind nslices idc offA offB t8 wp cip nrefs qpmin qpmax
 *                   pcm_permille intra_permille mvx mvy seed index out.yuv [recon_only
 *                   [lossless_permille [sp_slices [structure [chroma_format]]]]]
 * lossless_permille > 0 sets sps.qpprime_y_zero_transform_bypass_flag (the synthetic
 * pictures then hold TransformBypassModeFlag MBs, interpret_mb.cc:804).
 * structure 1 / 2 decodes a top / bottom FIELD picture of H MB rows (shr.field_pic_flag,
 * frame_mbs_only_flag 0): its references are field storable_pictures split from the synthetic
 * DPB frames of 2H rows (as dpb_split_field picture.cc:408-470 does), the coefficient push
 * takes the reference's own field scan (Transform::inverse_scan_* read field_pic_flag,
 * transform.cc:338-386), and deblock_filter runs on the field (exit_picture picture.cc:253).
 * chroma_format 3 decodes a 4:4:4 picture (sps.chroma_format_idc 3, High 4:4:4 Predictive): every
 * plane's coefficients go through coeff_luma_* / transform_luma_dc with its ColorPlane, as the
 * parser does for ChromaArrayType 3 (interpret_residual.cc), and the references are padded
 * with the luma pads, as pad_dec_picture does for 4:4:4 (picture.cc:207-232).
 * chroma_format 2 decodes a 4:2:2 picture (High 4:2:2, MbHeightC 16): the chroma DC levels go
 * through coeff_chroma_dc at the scan index the reference's own inverse_scan_chroma_dc maps to
 * their raster position (transform.cc:365-374), the AC levels of the 8 blocks per plane through
 * coeff_chroma_ac, and the references take the 4:2:2 chroma pads (picture.cc:27-29).
 * chroma_format 4 (H264R_SYNTH_CHROMA_400) decodes a 4:0:0 picture (High, ChromaArrayType 0): no chroma planes anywhere
 * (picture.cc:34, decoder.cc:199, deblock.cc:498,522); the output holds the luma plane alone.
 * Output: Y plane then Cb then Cr, 8-bit, unpadded.
 *
 * Timing mode (H264R_TIME_REPS=<n>): the reconstruction of the picture -- the
 * coefficient push (inverse scan + dequantisation), Decoder::decode of every MB and
 * deblock_filter -- runs n times back to back on one thread (every pass rewrites every
 * MB, so each pass decodes the same picture), and "ref_time <MBs> <seconds>" goes to
 * stderr.  The output file holds the last pass.
 */
#include "global.h"
#include "slice.h"
#include "dpb.h"
#include "macroblock.h"
#include "decoder.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" {
#include "h264r.h"
#include "h264r_synth.h"
}

extern void pad_buf(px_t* pImgBuf, int iWidth, int iHeight, int iStride, int iPadX, int iPadY);

using namespace vio::h264;

static void zigzag(int n, int* inv /* raster -> scan index */)
{
    /* frame zig-zag (spec Tables 8-12/8-13): anti-diagonals, odd ones top-right to bottom-left */
    int idx = 0;
    for (int s = 0; s <= 2 * (n - 1); ++s) {
        if (s & 1) {
            for (int x = (s < n ? s : n - 1); x >= 0 && s - x < n; --x) inv[(s - x) * n + x] = idx++;
        } else {
            for (int x = (s < n ? 0 : s - n + 1); x <= s && x < n; ++x) inv[(s - x) * n + x] = idx++;
        }
    }
}

int main(int argc, char** argv)
{
    if (argc < 21) {
        fprintf(stderr, "usage: %s W H kind nslices idc offA offB t8 wp cip nrefs qpmin qpmax pcm intra mvx mvy seed index out [recon_only]\n", argv[0]);
        return 2;
    }
    h264r_synth_cfg cfg;
    memset(&cfg, 0, sizeof(cfg));
    int k = 1;
    cfg.width_mbs = atoi(argv[k++]); cfg.height_mbs = atoi(argv[k++]);
    cfg.kind = atoi(argv[k++]); cfg.num_slices = atoi(argv[k++]);
    cfg.deblock_idc = atoi(argv[k++]); cfg.filter_offset_a = atoi(argv[k++]); cfg.filter_offset_b = atoi(argv[k++]);
    cfg.transform8x8 = atoi(argv[k++]); cfg.wp_mode = atoi(argv[k++]); cfg.constrained_intra = atoi(argv[k++]);
    cfg.num_refs = atoi(argv[k++]); cfg.qp_min = atoi(argv[k++]); cfg.qp_max = atoi(argv[k++]);
    cfg.pcm_permille = atoi(argv[k++]); cfg.intra_permille = atoi(argv[k++]);
    cfg.mv_range_x = atoi(argv[k++]); cfg.mv_range_y = atoi(argv[k++]);
    cfg.seed = strtoull(argv[k++], nullptr, 0);
    int index = atoi(argv[k++]);
    const char* out_path = argv[k++];
    bool recon_only = argc > k && atoi(argv[k]) != 0;
    if (argc > k + 1) cfg.lossless_permille = atoi(argv[k + 1]);
    if (argc > k + 2) cfg.sp_slices = atoi(argv[k + 2]);
    if (argc > k + 3) cfg.structure = atoi(argv[k + 3]);
    if (argc > k + 4) cfg.chroma_format = atoi(argv[k + 4]);
    /* argument 27: 1 + colour_plane_id of a separate-colour-plane (JV) frame: the synthetic picture is
       monochrome (4:0:0 records) and is decoded as that colour plane of a 4:4:4 frame
       (separate_colour_plane_flag, slice colour_plane_id); the other two planes are blank
       pictures whose filter changes nothing, and the output is the decoded plane after the
       reference's Deblock::deblock / make_frame_picture_JV (deblock.cc:555-579, 641-655) */
    const int jv = argc > k + 5 ? atoi(argv[k + 5]) : 0;
    const bool f444 = cfg.chroma_format == 3, f422 = cfg.chroma_format == 2, f400 = cfg.chroma_format == H264R_SYNTH_CHROMA_400;
    const int CW = f400 ? 0 : f444 ? 16 : 8, CH = f400 ? 0 : f444 || f422 ? 16 : 8;   /* chroma samples per MB */
    const bool fld = cfg.structure == H264R_TOP_FIELD || cfg.structure == H264R_BOTTOM_FIELD;
    if (jv && (!f400 || cfg.structure != H264R_FRAME || jv > 3)) { fprintf(stderr, "JV: 4:0:0 records of a frame\n"); return 2; }
    const int RW = jv ? 16 : CW, RH = jv ? 16 : CH;     /* the planes' chroma samples per MB (JV: 4:4:4) */
    /* MBAFF frame (argument 25 = 3): mb_data by MB address (pairs), mb.mb the storage position,
       field MBs predicting from the fields of the list's frames (get_ref_pic dpb.cc:1046-1055) */
    const bool mbaff = cfg.structure == H264R_MBAFF_FRAME;
    const PictureStructure pstruct = cfg.structure == H264R_TOP_FIELD ? TOP_FIELD
                                   : cfg.structure == H264R_BOTTOM_FIELD ? BOTTOM_FIELD : FRAME;

    const int W = cfg.width_mbs, H = cfg.height_mbs, NMB = W * H, W4 = W * 4, PL = W4 * H * 4;
    std::vector<h264r_mb> mbs(NMB);
    std::vector<int16_t> levels((size_t)NMB * H264R_SYNTH_MAX_LEVELS_PER_MB_444);
    std::vector<uint32_t> mv(2 * (size_t)PL);
    std::vector<int8_t> ref_idx(2 * (size_t)PL);
    std::vector<h264r_slice> slices(cfg.num_slices);
    h264r_pic pic;
    int64_t nlev = 0;
    if (h264r_synth_picture(&cfg, index, mbs.data(), levels.data(), &nlev, mv.data(), ref_idx.data(),
                            slices.data(), &pic) != H264R_OK) {
        fprintf(stderr, "synth failed\n");
        return 3;
    }

    VideoParameters* vid = new VideoParameters();
    sps_t* sps = new sps_t();
    pps_t* pps = new pps_t();
    sps->profile_idc = f444 ? 244 : f422 ? 122 : 100; sps->level_idc = 51;
    sps->chroma_format_idc = f444 ? 3 : f422 ? 2 : f400 ? 0 : 1; sps->ChromaArrayType = sps->chroma_format_idc;
    if (jv) {                          /* interpret_rbsp.cc:100,123-127 */
        sps->profile_idc = 244; sps->chroma_format_idc = 3; sps->separate_colour_plane_flag = 1; sps->ChromaArrayType = 0;
    }
    sps->SubWidthC = f444 ? 1 : 2; sps->SubHeightC = CH == 8 ? 2 : 1; sps->MbWidthC = CW; sps->MbHeightC = CH;
    sps->BitDepthY = 8; sps->BitDepthC = 8;
    sps->frame_mbs_only_flag = !fld; sps->direct_8x8_inference_flag = 1;
    const int FH = fld ? 2 * H : H;                     /* FrameHeightInMbs */
    sps->PicWidthInMbs = W; sps->FrameHeightInMbs = FH;
    sps->PicWidthInSamplesL = W * 16; sps->PicWidthInSamplesC = W * CW;
    sps->PicHeightInMapUnits = H; sps->PicSizeInMapUnits = W * H;
    sps->qpprime_y_zero_transform_bypass_flag = cfg.lossless_permille > 0;
    /* H264R_QMATRIX=<file>: 6x16 + 6x64 int32 raster scaling lists, every one present in
     * the SPS (Transform::init then takes them as they are, transform.cc:183-214) */
    if (const char* qm = getenv("H264R_QMATRIX")) {
        FILE* f = fopen(qm, "rb");
        int32_t v[6 * 16 + 6 * 64];
        if (!f || fread(v, sizeof(v), 1, f) != 1) { fprintf(stderr, "cannot read %s\n", qm); return 2; }
        fclose(f);
        sps->seq_scaling_matrix_present_flag = 1;
        for (int i = 0; i < 12; ++i) sps->seq_scaling_list_present_flag[i] = 1;
        for (int i = 0; i < 6; ++i) {
            sps->UseDefaultScalingMatrix4x4Flag[i] = 0; sps->UseDefaultScalingMatrix8x8Flag[i] = 0;
            for (int k = 0; k < 16; ++k) sps->ScalingList4x4[i][k] = v[i * 16 + k];
            for (int k = 0; k < 64; ++k) sps->ScalingList8x8[i][k] = v[96 + i * 64 + k];
        }
    }
    pps->entropy_coding_mode_flag = 0;
    pps->weighted_pred_flag = cfg.kind == H264R_SYNTH_P && cfg.wp_mode == 1;
    pps->weighted_bipred_idc = cfg.kind == H264R_SYNTH_B ? cfg.wp_mode : 0;
    pps->constrained_intra_pred_flag = cfg.constrained_intra;
    pps->transform_8x8_mode_flag = cfg.transform8x8;
    pps->deblocking_filter_control_present_flag = 1;
    vid->active_sps = sps; vid->active_pps = pps;
    vid->no_reference_picture = nullptr;

    /* DPB: reference pictures, padded like exit_picture (picture.cc:258-259); a field picture's
       references are the fields of the DPB frames, refs[2 s + bottom] */
    const int nfr = h264r_synth_ref_frames(&cfg);
    std::vector<storable_picture*> refs(fld ? 2 * nfr : nfr);
    std::vector<uint8_t> ty(W * 16 * FH * 16), tu(W * RW * FH * RH + 1), tv(W * RW * FH * RH + 1);
    for (int s = 0; s < nfr; ++s) {
        h264r_synth_refpic_fmt(cfg.seed, s, W, FH, jv ? 3 : cfg.chroma_format, ty.data(), tu.data(), tv.data());
        for (int f = 0; f < (fld ? 2 : 1); ++f) {
            storable_picture* r = new storable_picture(vid, fld ? (f ? BOTTOM_FIELD : TOP_FIELD) : FRAME,
                                                       W * 16, FH * 16, W * RW, FH * RH, 1);
            const int step = fld ? 2 : 1;                /* dpb_split_field: every second row */
            for (int y = 0; y < H * 16; ++y) for (int x = 0; x < W * 16; ++x) r->imgY[y][x] = ty[(y * step + f) * W * 16 + x];
            for (int y = 0; y < H * RH; ++y) for (int x = 0; x < W * RW; ++x) {
                r->imgUV[0][y][x] = tu[(y * step + f) * W * RW + x];
                r->imgUV[1][y][x] = tv[(y * step + f) * W * RW + x];
            }
            pad_buf(*r->imgY, W * 16, H * 16, r->iLumaStride, MCBUF_LUMA_PAD_X, MCBUF_LUMA_PAD_Y);
            if (!f400 || jv) {
                pad_buf(*r->imgUV[0], W * RW, H * RH, r->iChromaStride, r->iChromaPadX, r->iChromaPadY);
                pad_buf(*r->imgUV[1], W * RW, H * RH, r->iChromaStride, r->iChromaPadX, r->iChromaPadY);
            }
            r->poc = r->frame_poc = r->top_poc = r->bottom_poc = h264r_synth_slot_poc(s) + f;
            r->is_long_term = 0; r->used_for_reference = 1;
            refs[fld ? 2 * s + f : s] = r;
        }
        if (mbaff) {                                     /* the frame's two fields (dpb_split_field) */
            storable_picture* fr = refs[s];
            for (int f = 0; f < 2; ++f) {
                storable_picture* r = new storable_picture(vid, f ? BOTTOM_FIELD : TOP_FIELD, W * 16, FH * 16, W * CW, FH * CH, 1);   /* halved by the ctor */
                for (int y = 0; y < FH * 8; ++y) for (int x = 0; x < W * 16; ++x) r->imgY[y][x] = ty[(2 * y + f) * W * 16 + x];
                for (int y = 0; y < FH * CH / 2; ++y) for (int x = 0; x < W * CW; ++x) {
                    r->imgUV[0][y][x] = tu[(2 * y + f) * W * CW + x];
                    r->imgUV[1][y][x] = tv[(2 * y + f) * W * CW + x];
                }
                pad_buf(*r->imgY, W * 16, FH * 8, r->iLumaStride, MCBUF_LUMA_PAD_X, MCBUF_LUMA_PAD_Y);
                pad_buf(*r->imgUV[0], W * CW, FH * CH / 2, r->iChromaStride, r->iChromaPadX, r->iChromaPadY);
                pad_buf(*r->imgUV[1], W * CW, FH * CH / 2, r->iChromaStride, r->iChromaPadX, r->iChromaPadY);
                r->poc = r->frame_poc = r->top_poc = r->bottom_poc = h264r_synth_slot_poc(s) + f;
                r->is_long_term = 0; r->used_for_reference = 1;
                r->frame = fr;
                (f ? fr->bottom_field : fr->top_field) = r;
            }
        }
    }
    /* RefPicList entry -> storable_picture (include/h264r.h: slot | H264R_REF_BOTTOM for fields) */
    auto ref_of = [&](int v) { return fld ? refs[2 * (v & 31) + ((v & H264R_REF_BOTTOM) ? 1 : 0)] : refs[v]; };

    storable_picture* dec = new storable_picture(vid, pstruct, W * 16, FH * 16, W * RW, FH * RH, 1);
    dec->sps = sps; dec->pps = pps;
    dec->used_for_reference = 1;
    dec->poc = dec->frame_poc = pic.poc;
    vid->dec_picture = dec;
    mb_t* mb_data = new mb_t[NMB];
    memset((void*)mb_data, 0, sizeof(mb_t) * NMB);
    for (int a = 0; a < NMB; ++a) mb_data[a].slice_nr = -1;   /* reset_mbs, slice_data.cc:53-58 */
    vid->mb_data = mb_data;

    std::vector<slice_t*> sl(cfg.num_slices);
    for (int s = 0; s < cfg.num_slices; ++s) {
        const h264r_slice& c = slices[s];
        slice_t* x = new slice_t();
        x->p_Vid = vid; x->active_sps = sps; x->active_pps = pps;
        shr_t& h = x->header;
        h.slice_type = c.slice_type;
        h.structure = pstruct; h.MbaffFrameFlag = mbaff; h.field_pic_flag = fld;
        h.colour_plane_id = (uint8_t)(jv ? jv - 1 : 0);
        h.bottom_field_flag = pstruct == BOTTOM_FIELD;
        h.PicHeightInMbs = H; h.PicHeightInSamplesL = H * 16; h.PicHeightInSamplesC = H * CH;
        h.PicSizeInMbs = W * H;
        h.disable_deblocking_filter_idc = c.deblock_idc;
        h.FilterOffsetA = c.filter_offset_a; h.FilterOffsetB = c.filter_offset_b;
        h.luma_log2_weight_denom = c.luma_log2_wd; h.chroma_log2_weight_denom = c.chroma_log2_wd;
        h.PicOrderCnt = h.TopFieldOrderCnt = h.BottomFieldOrderCnt = pic.poc;
        h.direct_spatial_mv_pred_flag = 0;
        h.QsY = (int8_t)c.qs_y; h.sp_for_switch_flag = c.sp_switch;      /* SP slices (interpret_rbsp.cc:738-748) */
        for (int l = 0; l < 2; ++l)
            for (int pl = 0; pl < 3; ++pl) {
                h.pred_weight_l[l][pl].resize(H264R_MAX_REFS);
                for (int i = 0; i < H264R_MAX_REFS; ++i) {
                    h.pred_weight_l[l][pl][i].weight_flag = 1;
                    h.pred_weight_l[l][pl][i].weight = c.wp_weight[l][i][pl];
                    h.pred_weight_l[l][pl][i].offset = c.wp_offset[l][i][pl];
                }
            }
        for (int l = 0; l < 2; ++l) {
            x->RefPicSize[l] = (char)c.num_ref[l];
            for (int i = 0; i < c.num_ref[l]; ++i) x->RefPicList[l][i] = ref_of(c.ref_slot[l][i]);
        }
        x->current_slice_nr = (short)s;
        x->dec_picture = dec;
        x->neighbour.mb_data = mb_data;
        x->decoder.init(*x);
        x->decoder.assign_quant_params(*x);
        dec->slice_headers.push_back(x);
        sl[s] = x;
    }

    /* motion field (written by the parser, interpret_mb.cc:583-623) */
    for (int y4 = 0; y4 < H * 4; ++y4)
        for (int x4 = 0; x4 < W4; ++x4) {
            int idx = y4 * W4 + x4;
            const h264r_mb& m = mbs[(y4 / 4) * W + x4 / 4];
            pic_motion_params& p = dec->mv_info[y4][x4];
            p.slice_no = (uint8_t)m.slice;
            const bool fmb = mbaff && (m.flags & H264R_MBF_FIELD);
            const int mbot = (y4 / 4) & 1;
            for (int l = 0; l < 2; ++l) {
                int r = ref_idx[(size_t)l * PL + idx];
                uint32_t v = mv[(size_t)l * PL + idx];
                p.ref_idx[l] = (char)r;
                p.mv[l].mv_x = (int16_t)(v & 0xFFFF);
                p.mv[l].mv_y = (int16_t)(v >> 16);
                /* get_ref_pic (dpb.cc:1046-1055), as the parser stores it (interpret_mb.cc:617-620) */
                p.ref_pic[l] = r < 0 ? nullptr : !fmb ? sl[m.slice]->RefPicList[l][r]
                             : (mbot == r % 2 ? sl[m.slice]->RefPicList[l][r / 2]->top_field
                                              : sl[m.slice]->RefPicList[l][r / 2]->bottom_field);
            }
        }

    int inv4[16], inv8[64], inv4f[16], inv8f[64];
    zigzag(4, inv4);
    zigzag(8, inv8);
    if (mbaff) {                     /* a field MB's scans (transform.cc:344-357: mb_field_decoding_flag) */
        mb_t probe;
        memset((void*)&probe, 0, sizeof(probe));
        probe.p_Slice = sl[0];
        probe.mb_field_decoding_flag = 1;
        for (int t8 = 0; t8 < 2; ++t8) {
            probe.transform_size_8x8_flag = t8;
            for (int k = 0; k < (t8 ? 64 : 16); ++k) {
                const pos_t pos = sl[0]->decoder.transform->inverse_scan_luma_ac(&probe, k);
                (t8 ? inv8f : inv4f)[pos.y * (t8 ? 8 : 4) + pos.x] = k;
            }
        }
    }
    if (fld) {
        /* the field scans (Tables 8-13 / 8-14) as the reference maps them: raster position of
           each scan index from its own Transform::inverse_scan_luma_ac on a field slice */
        mb_t probe;
        memset((void*)&probe, 0, sizeof(probe));
        probe.p_Slice = sl[0];
        for (int t8 = 0; t8 < 2; ++t8) {
            probe.transform_size_8x8_flag = t8;
            for (int k = 0; k < (t8 ? 64 : 16); ++k) {
                const pos_t pos = sl[0]->decoder.transform->inverse_scan_luma_ac(&probe, k);
                (t8 ? inv8 : inv4)[pos.y * (t8 ? 8 : 4) + pos.x] = k;
            }
        }
        /* H264R_PRINT_FIELD_SCANS: the field scans as raster index per scan position, for the
           repo's parser tables (tools/gen_parser_tables.py via tests/golden/make_cabac_tables.py) */
        if (getenv("H264R_PRINT_FIELD_SCANS")) {
            int s4[16], s8[64];
            for (int r = 0; r < 16; ++r) s4[inv4[r]] = r;
            for (int r = 0; r < 64; ++r) s8[inv8[r]] = r;
            printf("{\"field_scan4x4\": [");
            for (int k = 0; k < 16; ++k) printf("%s%d", k ? ", " : "", s4[k]);
            printf("], \"field_scan8x8\": [");
            for (int k = 0; k < 64; ++k) printf("%s%d", k ? ", " : "", s8[k]);
            printf("]}\n");
            return 0;
        }
    }

    /* 4:2:2 chroma DC: the scan index of each raster position of the 2x4 matrix, from the
       reference's own inverse_scan_chroma_dc */
    int dc422[8] = {0};
    if (f422) {
        mb_t probe;
        memset((void*)&probe, 0, sizeof(probe));
        probe.p_Slice = sl[0];
        for (int k = 0; k < 8; ++k) {
            const pos_t pos = sl[0]->decoder.transform->inverse_scan_chroma_dc(&probe, k);
            dc422[pos.y * 2 + pos.x] = k;
        }
    }

    const char* reps_env = getenv("H264R_TIME_REPS");
    const int reps = reps_env ? atoi(reps_env) : 1;
    /* every pass starts from the parser's state of mb_data (reset_mbs) */
    std::vector<char> mb_pristine(sizeof(mb_t) * NMB);
    memcpy(mb_pristine.data(), (void*)mb_data, mb_pristine.size());
    double sec = 0;
    for (int rep = 0; rep < reps; ++rep) {
    if (rep) memcpy((void*)mb_data, mb_pristine.data(), mb_pristine.size());
    const auto t0 = std::chrono::steady_clock::now();
    for (int a = 0; a < NMB; ++a) {
        /* MBAFF: MB address a is pair a / 2's top or bottom MB, stored at row 2 pair_row + a % 2 */
        const int si = mbaff ? ((a / 2) / W * 2 + a % 2) * W + (a / 2) % W : a;
        const h264r_mb& c = mbs[si];
        slice_t& s = *sl[c.slice];
        mb_t& mb = mb_data[a];
        mb.p_Slice = &s; mb.mbAddrX = a; mb.mb.x = si % W; mb.mb.y = si / W;
        mb.slice_nr = (short)c.slice;
        mb.is_intra_block = (c.flags & H264R_MBF_INTRA) != 0;
        mb.mb_type = c.mb_type;
        mb.transform_size_8x8_flag = (c.flags & H264R_MBF_T8x8) != 0;
        mb.mb_field_decoding_flag = mbaff && (c.flags & H264R_MBF_FIELD);
        if (mbaff) dec->motion.mb_field_decoding_flag[a] = mb.mb_field_decoding_flag;
        const int* sc4 = mb.mb_field_decoding_flag ? inv4f : inv4;
        const int* sc8 = mb.mb_field_decoding_flag ? inv8f : inv8;
        for (int b = 0; b < 16; ++b) mb.Intra4x4PredMode[b] = (c.ipred[b >> 1] >> ((b & 1) * 4)) & 15;
        for (int b = 0; b < 4; ++b) mb.Intra8x8PredMode[b] = (c.ipred[b >> 1] >> ((b & 1) * 4)) & 15;
        mb.Intra16x16PredMode = c.i16_mode;
        mb.intra_chroma_pred_mode = c.chroma_mode;
        mb.CodedBlockPatternLuma = c.cbp & 15;
        mb.CodedBlockPatternChroma = c.cbp >> 4;
        mb.QpY = c.qp_y; mb.QpC[0] = c.qp_c[0]; mb.QpC[1] = c.qp_c[1];
        mb.QsC[0] = slices[c.slice].qs_c[0]; mb.QsC[1] = slices[c.slice].qs_c[1];   /* interpret_mb.cc:799-801 */
        s.parser.QpY = c.qp_y;                   /* itrans_sp reads the parser's running QpY (transform.cc:1138) */
        mb.qp_scaled[0] = c.qp_scaled[0]; mb.qp_scaled[1] = c.qp_scaled[1]; mb.qp_scaled[2] = c.qp_scaled[2];
        /* interpret_mb.cc:804 */
        mb.TransformBypassModeFlag = sps->qpprime_y_zero_transform_bypass_flag && mb.qp_scaled[0] == 0;
        if (mb.TransformBypassModeFlag != ((c.flags & H264R_MBF_BYPASS) != 0) && c.mb_type != H264R_I_PCM) {
            fprintf(stderr, "bypass flag mismatch at MB %d\n", si);
            return 4;
        }
        memset(mb.cbp_blks, 0, sizeof(mb.cbp_blks));
        /* partition shape for the reference's own partition walk (decoder.cc:217-254) */
        if (!mb.is_intra_block) {
            for (int b8 = 0; b8 < 4; ++b8) {
                int bx = (b8 & 1) * 2 + mb.mb.x * 4, by = (b8 >> 1) * 2 + mb.mb.y * 4;
                const pic_motion_params& t = dec->mv_info[by][bx];
                mb.SubMbPredMode[b8] = (t.ref_idx[0] >= 0 && t.ref_idx[1] >= 0) ? 2 : (t.ref_idx[0] >= 0 ? 0 : 1);
                if (c.mb_type >= 1 && c.mb_type <= 3) mb.SubMbType[b8] = c.mb_type;
                else if (c.mb_type == 4) {
                    auto same = [&](int dx0, int dy0, int dx1, int dy1) {
                        const pic_motion_params& u = dec->mv_info[by + dy0][bx + dx0];
                        const pic_motion_params& v = dec->mv_info[by + dy1][bx + dx1];
                        return u.ref_idx[0] == v.ref_idx[0] && u.ref_idx[1] == v.ref_idx[1] &&
                               u.mv[0] == v.mv[0] && u.mv[1] == v.mv[1];
                    };
                    bool rows = same(0, 0, 1, 0) && same(0, 1, 1, 1);   /* each row uniform -> 8x4 */
                    bool cols = same(0, 0, 0, 1) && same(1, 0, 1, 1);   /* each col uniform -> 4x8 */
                    mb.SubMbType[b8] = (rows && cols) ? 4 : rows ? 5 : cols ? 6 : 7;
                } else mb.SubMbType[b8] = 0;
            }
        }

        /* coefficient push, slice_data.cc:496-503 reset protocol then the parser's calls */
        Transform* tr = s.decoder.transform;
        memset(tr->cof, 0, sizeof(tr->cof));
        const int16_t* lv = levels.data() + c.coef_off;
        if (c.mb_type == H264R_I_PCM) {
            const uint8_t* raw = (const uint8_t*)lv;
            for (int y = 0; y < 16; ++y) for (int x = 0; x < 16; ++x) tr->cof[0][y][x] = raw[y * 16 + x];
            for (int q = 0; q < 2; ++q)
                for (int y = 0; y < CH; ++y) for (int x = 0; x < CW; ++x)
                    tr->cof[1 + q][y][x] = raw[256 + q * CW * CH + y * CW + x];
            mb.cbp_blks[0] = 0xFFFF;
        } else {
            int cbpl = c.cbp & 15, cbpc = c.cbp >> 4;
            const int16_t* p = lv;
            const int16_t* b8p[4] = {nullptr, nullptr, nullptr, nullptr};
            for (int q = 0; q < 4; ++q) if (cbpl & (1 << q)) { b8p[q] = p; p += 64; }
            const int nb = f422 ? 8 : 4;                /* chroma 4x4 blocks per plane */
            const int16_t *cac = nullptr, *ldc = nullptr, *cdc = nullptr;
            if (f422) {                                 /* include/h264r.h: luma, then chroma AC, DC */
                if (c.mb_type == H264R_I_16x16) { ldc = p; p += 16; }
                if (cbpc == 2) { cac = p; p += 256; }
                if (cbpc) { cdc = p; p += 16; }
            } else {
                if (cbpc == 2) { cac = p; p += 128; }
                if (c.mb_type == H264R_I_16x16) { ldc = p; p += 16; }
                if (cbpc) { cdc = p; p += 8; }
            }
            /* a luma-like block (every plane of a 4:4:4 MB: the coded 8x8 blocks, then the I16 DC) */
            auto push_luma = [&](ColorPlane pl, const int16_t* const* b8, const int16_t* dc) {
                if (dc) {
                    for (int pos = 0; pos < 16; ++pos)
                        if (dc[pos]) s.decoder.coeff_luma_dc(&mb, pl, 0, 0, sc4[pos], dc[pos]);
                    s.decoder.transform_luma_dc(&mb, pl);
                }
                for (int q = 0; q < 4; ++q) {
                    if (!b8[q]) continue;
                    if (!mb.transform_size_8x8_flag) {
                        for (int b4 = 0; b4 < 4; ++b4) {
                            int x0 = (q & 1) * 2 + (b4 & 1), y0 = (q >> 1) * 2 + (b4 >> 1);
                            for (int pos = 0; pos < 16; ++pos) {
                                int v = b8[q][b4 * 16 + pos];
                                if (v) s.decoder.coeff_luma_ac(&mb, pl, x0, y0, sc4[pos], v);
                            }
                        }
                    } else {
                        int x0 = (q & 1) * 2, y0 = (q >> 1) * 2;
                        for (int pos = 0; pos < 64; ++pos) {
                            int v = b8[q][pos];
                            if (v) s.decoder.coeff_luma_ac(&mb, pl, x0, y0, sc8[pos], v);
                        }
                    }
                }
            };
            push_luma(PLANE_Y, b8p, ldc);
            for (int pl = 1; f444 && pl <= 2; ++pl) {
                const int16_t* cb8[4] = {nullptr, nullptr, nullptr, nullptr};
                for (int q = 0; q < 4; ++q) if (cbpl & (1 << q)) { cb8[q] = p; p += 64; }
                const int16_t* cdcp = nullptr; if (c.mb_type == H264R_I_16x16) { cdcp = p; p += 16; }
                push_luma((ColorPlane)pl, cb8, cdcp);
            }
            if (cbpc) {
                for (int pl = 1; pl <= 2; ++pl) {
                    for (int q = 0; q < nb; ++q)
                        if (cdc[(pl - 1) * nb + q])
                            s.decoder.coeff_chroma_dc(&mb, (ColorPlane)pl, 0, 0, f422 ? dc422[q] : q, cdc[(pl - 1) * nb + q]);
                    s.decoder.transform_chroma_dc(&mb, (ColorPlane)pl);
                }
            }
            if (cac) {
                for (int pl = 1; pl <= 2; ++pl)
                    for (int b = 0; b < nb; ++b)
                        for (int pos = 1; pos < 16; ++pos) {
                            int v = cac[(pl - 1) * nb * 16 + b * 16 + pos];
                            if (v) s.decoder.coeff_chroma_ac(&mb, (ColorPlane)pl, b % 2, b / 2, sc4[pos], v);
                        }
            }
        }
        if ((uint16_t)mb.cbp_blks[0] != c.cbp_blks) {
            fprintf(stderr, "cbp_blks mismatch at MB %d: reference %04x synth %04x\n", si, (unsigned)mb.cbp_blks[0], c.cbp_blks);
            return 4;
        }
        static const char* dump = getenv("H264R_DUMP_MB");
        if (dump && atoi(dump) == a) {
            int x0 = mb.mb.x * 16 - 1, y0 = mb.mb.y * 16;
            fprintf(stderr, "left column x=%d:", x0);
            for (int y = 0; y < 16 && x0 >= 0; ++y) fprintf(stderr, " %d", dec->imgY[y0 + y][x0]);
            fprintf(stderr, "\ncof (dequantised) plane 0:\n");
            for (int y = 0; y < 16; ++y) { for (int x = 0; x < 16; ++x) fprintf(stderr, "%6d", tr->cof[0][y][x]); fprintf(stderr, "\n"); }
        }
        s.decoder.decode(mb);
        if (dump && atoi(dump) == a) {
            fprintf(stderr, "mb_pred plane 0:\n");
            for (int y = 0; y < 16; ++y) { for (int x = 0; x < 16; ++x) fprintf(stderr, "%4d", s.mb_pred[0][y][x]); fprintf(stderr, "\n"); }
        }
    }
    if (jv) {
        /* the frame's other two colour planes: blank pictures with the decoded plane's slice headers
           (Deblock::deblock gates every plane on plane 0's slices, :632-640) and intra MBs of QP 0,
           whose edges the filter leaves alone (alpha 0) */
        for (int k = 0; k < 3; ++k) {
            if (k == jv - 1) { vid->dec_picture_JV[k] = dec; vid->mb_data_JV[k] = mb_data; continue; }
            storable_picture* dp = new storable_picture(vid, FRAME, W * 16, H * 16, W * 16, H * 16, 1);
            dp->sps = sps; dp->pps = pps; dp->used_for_reference = 1;
            mb_t* md = new mb_t[NMB];
            memset((void*)md, 0, sizeof(mb_t) * NMB);
            for (slice_t* x0 : sl) {
                slice_t* x = new slice_t();
                x->p_Vid = vid; x->active_sps = sps; x->active_pps = pps;
                x->header = x0->header;
                x->header.colour_plane_id = (uint8_t)k;
                x->dec_picture = dp;
                x->neighbour.mb_data = md;
                dp->slice_headers.push_back(x);
            }
            for (int a = 0; a < NMB; ++a) {
                md[a].p_Slice = dp->slice_headers[mbs[a].slice]; md[a].mbAddrX = a; md[a].mb.x = a % W; md[a].mb.y = a / W;
                md[a].slice_nr = (short)mbs[a].slice; md[a].is_intra_block = 1; md[a].mb_type = H264R_I_16x16;
            }
            vid->dec_picture_JV[k] = dp; vid->mb_data_JV[k] = md;
        }
        vid->dec_picture = vid->dec_picture_JV[0];
    }
    /* MBAFF: the loop filter's MbAffPostProc (deblock.cc:596-629) interleaves the field MBs; the
       reconstruction alone is that with every slice's filter off (:631-640) */
    if (recon_only && (mbaff || jv))
        for (int k = 0; k < (jv ? 3 : 1); ++k)
            for (slice_t* x : (jv ? vid->dec_picture_JV[k]->slice_headers : dec->slice_headers)) x->header.disable_deblocking_filter_idc = 1;
    /* JV: make_frame_picture_JV (:555-579) moves planes 1 and 2 into the frame's imgUV */
    storable_picture* jv_frame = jv ? vid->dec_picture_JV[0] : nullptr;
    if (!recon_only || mbaff || jv) sl[0]->decoder.deblock_filter(*sl[0]);
    if (jv) {
        px_t** plane = jv == 1 ? jv_frame->imgY : jv_frame->imgUV[jv - 2];
        FILE* f = fopen(out_path, "wb");
        if (!f) return 5;
        std::vector<uint8_t> row(W * 16);
        for (int y = 0; y < H * 16; ++y) {
            for (int x = 0; x < W * 16; ++x) row[x] = (uint8_t)plane[y][x];
            fwrite(row.data(), 1, W * 16, f);
        }
        fclose(f);
        return 0;
    }
    sec += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    if (reps_env) {
        fprintf(stderr, "ref_time %lld %.6f\n", (long long)NMB * reps, sec);
    }

    FILE* f = fopen(out_path, "wb");
    if (!f) return 5;
    std::vector<uint8_t> row(W * 16);
    for (int y = 0; y < H * 16; ++y) {
        for (int x = 0; x < W * 16; ++x) {
            if (dec->imgY[y][x] > 255) { fprintf(stderr, "sample > 255 at Y(%d,%d)\n", x, y); return 6; }
            row[x] = (uint8_t)dec->imgY[y][x];
        }
        fwrite(row.data(), 1, W * 16, f);
    }
    for (int q = 0; q < 2; ++q)
        for (int y = 0; y < H * CH; ++y) {
            for (int x = 0; x < W * CW; ++x) {
                if (dec->imgUV[q][y][x] > 255) { fprintf(stderr, "sample > 255 at C%d(%d,%d)\n", q, x, y); return 6; }
                row[x] = (uint8_t)dec->imgUV[q][y][x];
            }
            fwrite(row.data(), 1, W * CW, f);
        }
    fclose(f);
    return 0;
}
