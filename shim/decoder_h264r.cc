/*
 * decoder_h264r.cc -- drop-in replacement of the reference's decoder/decoder.cc.
 *
 * luuvish/arrow-h264 reaches macroblock reconstruction only through
 * class vio::h264::Decoder (src/codec/h264/decoder/decoder.h:301-338).  This file
 * defines every public method of that class with its unchanged signature and routes
 * the reconstruction to the C ABI of include/h264r.h (the MI355X kernels of
 * libh264r.so, or any other implementation of that ABI).  A maintainer builds the
 * reference with this file instead of decoder/decoder.cc; nothing else changes: the
 * parser still pushes coefficients through coeff_* during residual parsing
 * (interpret_residual.cc:159-170, 405-415, 430, 475), the MB loop still calls decode(mb)
 * (slice_data.cc:646) and exit_picture still calls deblock_filter (picture.cc:253).
 *
 *   reference (decoder.cc)                 here
 *   Decoder() / ~Decoder()  :35-49          the CPU engines stay (ERC get_block_luma,
 *                                           the parser's access to transform->cof)
 *   init(slice)             :52-57          records the slice (type, deblocking control,
 *                                           weights, RefPicList -> DPB slots)
 *   assign_quant_params     :59-62          Transform::init + set_quant restated: qmatrix
 *                                           with fall-back rules A/B (transform.cc:173-257)
 *                                           -> h264r_quant_init_lists
 *   coeff_luma_dc/ac, coeff_chroma_dc/ac    the RAW level at its raster position in cof
 *                           :81-96          (inverse scan of transform.cc:339-386), the
 *                                           cbp_blks bits of coeff_luma_ac (:431-436);
 *                                           dequantisation runs on the GPU
 *   transform_luma_dc / chroma_dc :98-105   nothing (the DC transforms run on the GPU)
 *   decode(mb)              :65-79          snapshot of the MB: h264r_mb record, its level
 *                                           block, its 16 motion entries per list; keeps
 *                                           the is_reset_coeff{,_cr} side effects of
 *                                           decoder.cc:196-197, 205-206, 260-261 and
 *                                           transform.cc:1075-1076, 1093-1094
 *   deblock_filter(slice)   :107-110        h264r_picture_begin + h264r_mb_submit of every
 *                                           MB + h264r_picture_end: reconstruction and
 *                                           deblocking of the whole picture, planes copied
 *                                           back into dec_picture->imgY/imgUV (8 -> px_t);
 *                                           a reference picture stays on the device as a
 *                                           DPB slot for the motion compensation of later
 *                                           pictures
 *   get_block_luma          :112-116        unchanged CPU path (error concealment only)
 *
 * Reconstruction is deferred to picture end: the parser never reads reconstructed
 * samples (only syntax and mv_info), so the result is the same.
 *
 * MBAFF frames (MbaffFrameFlag): every MB is staged at its storage position mb_t::mb with its
 * mb_field_decoding_flag (H264R_MBF_FIELD) and the picture goes in as H264R_MBAFF_FRAME.
 * Field pictures (PAFF, field_pic_flag): the reference
 * decodes a field into a field storable_picture of half the frame's rows and deblocks it on
 * its own (exit_picture picture.cc:239-269), splits decoded frames into field views
 * (dpb_split_field picture.cc:408-470) and combines decoded field pairs into frames
 * (dpb_combine_field_yuv :573-590).  On the device a DPB slot is a frame: a decoded field is
 * kept in its parity's rows of a slot -- the second field of a pair in its first field's slot
 * (the pairing test of store_picture dpb.cc:903-912) -- and a reference list entry names a
 * slot (frame) or a slot's field (slot | H264R_REF_BOTTOM), found from whichever of a frame
 * store's pictures (frame, top_field, bottom_field) the shim decoded.
 * 4:2:2 (chroma_format_idc 2, MbHeightC 16; frame pictures): the level block takes the 4:2:2
 * layout of include/h264r.h (luma, then chroma AC of 8 blocks per plane, then the 2x4 DC
 * matrix -- coeff_chroma_dc left each DC level at its raster position, transform.cc:365-374).
 * 4:4:4 (chroma_format_idc 3, separate_colour_plane_flag 0; frame pictures): Cb and Cr are coded
 * like luma (coeff_luma_* with their ColorPlane), so the level block is three luma-like blocks
 * (include/h264r.h), and decode() leaves both coefficient-reset flags cleared (decoder.cc:72-76).
 * Errors: a status other than H264R_OK goes through the reference's own error()
 * (ldecod.cc:33-48), its convention for fatal conditions.
 */
#include "global.h"
#include "dpb.h"
#include "slice.h"
#include "macroblock.h"
#include "decoder.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

extern "C" {
#include "h264r.h"
}

namespace {

using namespace vio::h264;

// Flat and default scaling lists (Tables 7-3 / 7-4), raster order.
const int32_t FLAT16[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
                            16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
                            16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
                            16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16};
const int32_t DEF4_INTRA[16] = {6, 13, 20, 28, 13, 20, 28, 32, 20, 28, 32, 37, 28, 32, 37, 42};
const int32_t DEF4_INTER[16] = {10, 14, 20, 24, 14, 20, 24, 27, 20, 24, 27, 30, 24, 27, 30, 34};
const int32_t DEF8_INTRA[64] = {6, 10, 13, 16, 18, 23, 25, 27, 10, 11, 16, 18, 23, 25, 27, 29,
                                13, 16, 18, 23, 25, 27, 29, 31, 16, 18, 23, 25, 27, 29, 31, 33,
                                18, 23, 25, 27, 29, 31, 33, 36, 23, 25, 27, 29, 31, 33, 36, 38,
                                25, 27, 29, 31, 33, 36, 38, 40, 27, 29, 31, 33, 36, 38, 40, 42};
const int32_t DEF8_INTER[64] = {9, 13, 15, 17, 19, 21, 22, 24, 13, 13, 17, 19, 21, 22, 24, 25,
                                15, 17, 19, 21, 22, 24, 25, 27, 17, 19, 21, 22, 24, 25, 27, 28,
                                19, 21, 22, 24, 25, 27, 28, 30, 21, 22, 24, 25, 27, 28, 30, 32,
                                22, 24, 25, 27, 28, 30, 32, 33, 24, 25, 27, 28, 30, 32, 33, 35};

struct StagedMb {
    h264r_mb rec;
    std::vector<int16_t> levels;
    uint32_t mv[2][16];
    int8_t ref[2][16];
};

// Process-wide state: the reference keeps one Decoder per slice_t (slice.h:173), but one
// picture and one device context are shared by all of them.
struct Shim {
    h264r_ctx* ctx = nullptr;
    int ctx_w = 0, ctx_h = 0, ctx_cf = 0;   // the context's size and chroma_format_idc
    storable_picture* pic = nullptr;          // picture being staged
    std::vector<slice_t*> slices;             // its slices, in decoding order
    std::vector<h264r_slice> slice_tab;
    std::vector<StagedMb> mbs;
    std::vector<uint8_t> seen;
    h264r_quant quant;
    bool have_quant = false;
    // assign_quant_params runs while the slice header is parsed, before the picture it
    // belongs to is initialised (slice_header.cc:185 vs :195): its tables wait here until
    // init(slice) attaches the slice to its picture
    std::map<const slice_t*, h264r_quant> pending_quant;
    // decoded reference pictures resident on the device: their slot and the identity they had
    // when decoded (a picture the reference has freed may share its address with a later
    // split field or combined frame; the identity check keeps such an entry from matching)
    struct Resident { int slot; int structure; int poc; unsigned frame_num; };
    std::map<const storable_picture*, Resident> slot_of;
    int next_slot = 0;
    std::vector<uint8_t> y8, u8, v8;
};

Shim& shim()
{
    static Shim s;
    return s;
}

bool trace()
{
    static const bool t = getenv("H264R_SHIM_TRACE") != nullptr;
    return t;
}

void check(int st, const char* what)
{
    if (trace()) fprintf(stderr, "h264r shim: %s -> %d\n", what, st);
    if (st != H264R_OK) error(500, "h264r: %s failed: %s", what, h264r_strerror(st));
}

int slice_index(Shim& S, slice_t* sl)
{
    for (size_t i = 0; i < S.slices.size(); ++i)
        if (S.slices[i] == sl) return (int)i;
    return -1;
}

// The slot of a picture the shim decoded (NULL, the reference's no_reference_picture and
// pictures it did not decode: -1).
int decoded_slot(const Shim& S, const storable_picture* p)
{
    if (!p) return -1;
    auto it = S.slot_of.find(p);
    if (it == S.slot_of.end()) return -1;
    const Shim::Resident& r = it->second;
    if (r.structure != p->slice.structure || r.poc != p->poc || r.frame_num != p->frame_num) return -1;
    return r.slot;
}

// The device reference of a RefPicList entry: a frame picture's entry is a frame -- decoded as
// one, or combined from two decoded fields (its top_field / bottom_field); a field picture's is
// a field -- decoded as one, or split from a decoded frame (its `frame`) -- named by its slot and
// parity (include/h264r.h H264R_REF_BOTTOM).  -1 if none is resident.
int device_ref(const Shim& S, const storable_picture* p, bool field_pic)
{
    if (!p) return -1;
    const int st = p->slice.structure;
    int slot = -1;
    if (field_pic) {
        if (st == FRAME) return -1;
        slot = decoded_slot(S, p);
        if (slot < 0 && p->frame != p && p->frame && p->frame->slice.structure == FRAME) slot = decoded_slot(S, p->frame);
        return slot < 0 ? -1 : slot | (st == BOTTOM_FIELD ? H264R_REF_BOTTOM : 0);
    }
    if (st != FRAME) return -1;
    slot = decoded_slot(S, p);
    if (slot < 0 && p->top_field != p && p->top_field) slot = decoded_slot(S, p->top_field);
    if (slot < 0 && p->bottom_field != p && p->bottom_field) slot = decoded_slot(S, p->bottom_field);
    return slot;
}

// Start staging picture `pic` when the first of its slices arrives.
void begin_picture(Shim& S, slice_t& slice)
{
    storable_picture* pic = slice.dec_picture;
    if (S.pic == pic) return;
    const sps_t& sps = *slice.active_sps;
    const int cf = sps.chroma_format_idc;
    if (cf < 0 || cf > 3 || sps.separate_colour_plane_flag || sps.BitDepthY != 8 || (cf && sps.BitDepthC != 8))
        check(H264R_EUNSUPPORTED, "picture format (4:0:0, 4:2:0, 4:2:2 or 4:4:4 without separate planes, 8-bit)");
    if (slice.header.MbaffFrameFlag && cf != 1) check(H264R_EUNSUPPORTED, "MBAFF frames off 4:2:0");
    if (cf != 1 && slice.header.field_pic_flag) check(H264R_EUNSUPPORTED, "4:2:2 / 4:4:4 field pictures");
    // the context holds frames; a field picture is PicHeightInMbs = FrameHeightInMbs / 2 rows
    const int W = sps.PicWidthInMbs, H = sps.FrameHeightInMbs, PH = slice.header.PicHeightInMbs;
    if (!S.ctx || W > S.ctx_w || H > S.ctx_h || cf != S.ctx_cf) {
        if (S.ctx) h264r_destroy(S.ctx);
        S.ctx = nullptr;
        S.slot_of.clear();
        const char* dev = getenv("H264R_DEVICE");
        check(h264r_create(&S.ctx, dev ? atoi(dev) : 0, W, H, cf, 8), "h264r_create");
        S.ctx_w = W; S.ctx_h = H; S.ctx_cf = cf;
    }
    S.pic = pic;
    S.slices.clear();
    S.slice_tab.clear();
    S.mbs.assign((size_t)W * PH, StagedMb());
    S.seen.assign((size_t)W * PH, 0);
    S.have_quant = false;
}

// One h264r_slice from the slice header and the reference lists (slice.h:38-177).
h264r_slice slice_record(Shim& S, slice_t& slice)
{
    const shr_t& shr = slice.header;
    const pps_t& pps = *slice.active_pps;
    h264r_slice r;
    memset(&r, 0, sizeof(r));
    // MBAFF (include/h264r.h H264R_MBAFF_FRAME): a field MB's implicit weights (per-parity POCs) have
    // no place in h264r_slice; SP slices and lossless MBs are not on the MBAFF kernels
    if (shr.MbaffFrameFlag && ((shr.slice_type == B_slice && pps.weighted_bipred_idc == 2) || shr.slice_type == SP_slice))
        check(H264R_EUNSUPPORTED, "MBAFF slices with implicit weights / SP");
    // SI MBs go through mb_pred_inter in the reference with an out-of-range BLOCK_STEP row
    // (decoder.cc:141-146, 212-225): nothing defined to reproduce
    if (shr.slice_type == SI_slice) check(H264R_EUNSUPPORTED, "SI slices");
    r.slice_type = shr.slice_type;
    r.qs_y = (uint8_t)shr.QsY;                        // SP (interpret_rbsp.cc:738-748)
    r.sp_switch = shr.sp_for_switch_flag ? 1 : 0;
    r.deblock_idc = shr.disable_deblocking_filter_idc;
    r.filter_offset_a = shr.FilterOffsetA;
    r.filter_offset_b = shr.FilterOffsetB;
    const bool P = shr.slice_type == P_slice || shr.slice_type == SP_slice, B = shr.slice_type == B_slice;
    // inter_prediction.cc:62-63 (explicit) and :99-139 (implicit, B only)
    r.wp_mode = (pps.weighted_pred_flag && P) || (pps.weighted_bipred_idc == 1 && B) ? 1
              : (pps.weighted_bipred_idc == 2 && B) ? 2 : 0;
    r.luma_log2_wd = r.wp_mode == 1 ? shr.luma_log2_weight_denom : 5;
    r.chroma_log2_wd = r.wp_mode == 1 ? shr.chroma_log2_weight_denom : 5;
    for (int l = 0; l < 2; ++l) {
        const int n = (l == 0 ? (P || B) : B) ? std::min<int>(slice.RefPicSize[l], H264R_MAX_REFS) : 0;
        r.num_ref[l] = (uint8_t)n;
        for (int i = 0; i < H264R_MAX_REFS; ++i) {
            r.ref_slot[l][i] = -1;
            if (i < n && slice.RefPicList[l][i]) {
                // every picture of a reference list must be resident: a missing one would be
                // predicted as the reference's no_ref grey (inter_prediction.cc:164-167) --
                // fail loudly instead
                const int ref = device_ref(S, slice.RefPicList[l][i], shr.field_pic_flag);
                if (ref < 0) check(H264R_ESTATE, "reference picture not resident in a device DPB slot");
                r.ref_slot[l][i] = (int8_t)ref;
            }
            for (int pl = 0; pl < 3; ++pl) {
                const auto& v = shr.pred_weight_l[l][pl];
                if (r.wp_mode == 1 && i < (int)v.size()) {
                    r.wp_weight[l][i][pl] = v[i].weight;
                    r.wp_offset[l][i][pl] = v[i].offset;
                }
            }
        }
    }
    if (r.wp_mode == 2) {                                // implicit weights per (ref0, ref1)
        for (int i0 = 0; i0 < r.num_ref[0]; ++i0)
            for (int i1 = 0; i1 < r.num_ref[1]; ++i1) {
                const storable_picture* p0 = slice.RefPicList[0][i0];
                const storable_picture* p1 = slice.RefPicList[1][i1];
                int w1 = 32;
                if (p0 && p1) {
                    const int td = std::max(-128, std::min(127, p1->poc - p0->poc));
                    if (td != 0 && !p0->is_long_term && !p1->is_long_term) {
                        const int tb = std::max(-128, std::min(127, shr.PicOrderCnt - p0->poc));
                        const int tx = (16384 + std::abs(td / 2)) / td;
                        const int dsf = std::max(-1024, std::min(1023, (tx * tb + 32) >> 6));
                        w1 = dsf >> 2;
                        if (w1 < -64 || w1 > 128) w1 = 32;
                    }
                }
                r.implicit_w1[i0][i1] = (int16_t)w1;
            }
    }
    return r;
}

}  // namespace

namespace vio {
namespace h264 {

Decoder::Decoder() :
    intra_prediction { new IntraPrediction },
    inter_prediction { new InterPrediction },
    transform        { new Transform       },
    deblock          { new Deblock         }
{
}

Decoder::~Decoder()
{
    delete this->intra_prediction;
    delete this->inter_prediction;
    delete this->transform;
    delete this->deblock;
}

void Decoder::init(slice_t& slice)
{
    this->inter_prediction->init(slice);            // CPU engine kept for error concealment
    Shim& S = shim();
    begin_picture(S, slice);
    if (slice_index(S, &slice) < 0) {
        if ((int)S.slices.size() >= H264R_MAX_SLICES) check(H264R_EUNSUPPORTED, "slices per picture");
        S.slices.push_back(&slice);
        S.slice_tab.push_back(slice_record(S, slice));
        auto it = S.pending_quant.find(&slice);
        h264r_quant q;
        if (it != S.pending_quant.end()) q = it->second;
        else check(h264r_quant_init_flat(&q), "h264r_quant_init_flat");
        if (S.have_quant && memcmp(&S.quant, &q, sizeof(q)) != 0)
            check(H264R_EUNSUPPORTED, "scaling matrices differing between slices of one picture");
        S.quant = q;
        S.have_quant = true;
    }
}

void Decoder::assign_quant_params(slice_t& slice)
{
    // Transform::init (transform.cc:173-257): qmatrix[12] with the fall-back rules; the
    // dequantisation tables themselves (set_quant :259-302) are built by the library
    const sps_t& sps = *slice.active_sps;
    const pps_t& pps = *slice.active_pps;
    const int32_t* qm[12];
    if (!pps.pic_scaling_matrix_present_flag && !sps.seq_scaling_matrix_present_flag) {
        for (int i = 0; i < 12; ++i) qm[i] = FLAT16;
    } else {
        for (int i = 0; i < 12; ++i) qm[i] = i < 6 ? DEF4_INTRA : DEF8_INTRA;
        const int n = sps.chroma_format_idc != 3 ? 8 : 12;
        if (sps.seq_scaling_matrix_present_flag) {
            for (int i = 0; i < n; ++i) {
                if (i < 6) {
                    if (!sps.seq_scaling_list_present_flag[i])                        // rule A
                        qm[i] = i == 0 ? DEF4_INTRA : i == 3 ? DEF4_INTER : qm[i - 1];
                    else
                        qm[i] = sps.UseDefaultScalingMatrix4x4Flag[i] ? (i < 3 ? DEF4_INTRA : DEF4_INTER)
                                                                       : sps.ScalingList4x4[i];
                } else {
                    if (!sps.seq_scaling_list_present_flag[i])
                        qm[i] = i == 6 ? DEF8_INTRA : i == 7 ? DEF8_INTER : qm[i - 2];
                    else
                        qm[i] = sps.UseDefaultScalingMatrix8x8Flag[i - 6] ? ((i & 1) == 0 ? DEF8_INTRA : DEF8_INTER)
                                                                           : sps.ScalingList8x8[i - 6];
                }
            }
        }
        if (pps.pic_scaling_matrix_present_flag) {
            for (int i = 0; i < n; ++i) {
                if (i < 6) {
                    if (!pps.pic_scaling_list_present_flag[i]) {                    // rule B
                        if (i == 0) { if (!sps.seq_scaling_matrix_present_flag) qm[i] = DEF4_INTRA; }
                        else if (i == 3) { if (!sps.seq_scaling_matrix_present_flag) qm[i] = DEF4_INTER; }
                        else qm[i] = qm[i - 1];
                    } else
                        qm[i] = pps.UseDefaultScalingMatrix4x4Flag[i] ? (i < 3 ? DEF4_INTRA : DEF4_INTER)
                                                                       : pps.ScalingList4x4[i];
                } else {
                    if (!pps.pic_scaling_list_present_flag[i]) {
                        if (i == 6) { if (!sps.seq_scaling_matrix_present_flag) qm[i] = DEF8_INTRA; }
                        else if (i == 7) { if (!sps.seq_scaling_matrix_present_flag) qm[i] = DEF8_INTER; }
                        else qm[i] = qm[i - 2];
                    } else
                        qm[i] = pps.UseDefaultScalingMatrix8x8Flag[i - 6] ? ((i & 1) == 0 ? DEF8_INTRA : DEF8_INTER)
                                                                           : pps.ScalingList8x8[i - 6];
                }
            }
        }
        if (n == 8)                                                     // 4:2:0: lists 8..11 unused
            for (int i = 8; i < 12; ++i) qm[i] = qm[i - 2];
    }
    h264r_quant q;
    check(h264r_quant_init_lists(&q, qm), "h264r_quant_init_lists");
    this->transform->init(slice);                   // CPU engine kept in step (error concealment)
    shim().pending_quant[&slice] = q;
}

// Coefficient push (interpret_residual.cc:159-170, 405-415): the raw level at its raster
// position (the reference's Transform::coeff_* minus inverse_quantize, transform.cc:425-456).
void Decoder::coeff_luma_dc(mb_t* mb, ColorPlane pl, int x0, int y0, int runarr, int levarr)
{
    const pos_t& pos = this->transform->inverse_scan_luma_dc(mb, runarr);
    this->transform->cof[pl][pos.y * 4][pos.x * 4] = levarr;
}

void Decoder::coeff_luma_ac(mb_t* mb, ColorPlane pl, int x0, int y0, int runarr, int levarr)
{
    if (!mb->transform_size_8x8_flag)
        mb->cbp_blks[pl] |= ((uint64_t)0x01 << (y0 * 4 + x0));
    else
        mb->cbp_blks[pl] |= ((uint64_t)0x33 << (y0 * 4 + x0));
    const pos_t& pos = this->transform->inverse_scan_luma_ac(mb, runarr);
    this->transform->cof[pl][y0 * 4 + pos.y][x0 * 4 + pos.x] = levarr;
}

void Decoder::coeff_chroma_dc(mb_t* mb, ColorPlane pl, int x0, int y0, int runarr, int levarr)
{
    const pos_t& pos = this->transform->inverse_scan_chroma_dc(mb, runarr);
    this->transform->cof[pl][pos.y * 4][pos.x * 4] = levarr;
}

void Decoder::coeff_chroma_ac(mb_t* mb, ColorPlane pl, int x0, int y0, int runarr, int levarr)
{
    const pos_t& pos = this->transform->inverse_scan_chroma_ac(mb, runarr);
    this->transform->cof[pl][y0 * 4 + pos.y][x0 * 4 + pos.x] = levarr;
}

void Decoder::transform_luma_dc(mb_t*, ColorPlane)
{
}

void Decoder::transform_chroma_dc(mb_t*, ColorPlane)
{
}

void Decoder::decode(mb_t& mb)
{
    slice_t& slice = *mb.p_Slice;
    Shim& S = shim();
    const int (*cof)[16][16] = this->transform->cof;
    const int si = slice_index(S, &slice);
    if (si < 0) check(H264R_ESTATE, "decode() before init() of its slice");

    if (slice.header.slice_type == SP_slice && !mb.is_intra_block) {
        // itrans_sp_cr indexes LevelScale2 with QsC unreduced (transform.cc:1230,1235): the
        // reference reads past the table for QsC >= 6, so only QsC < 6 has defined output
        if (mb.QsC[0] >= 6 || mb.QsC[1] >= 6 || mb.QsC[0] < 0 || mb.QsC[1] < 0)
            check(H264R_EUNSUPPORTED, "SP slice with QsC >= 6");
        if (mb.transform_size_8x8_flag) check(H264R_EUNSUPPORTED, "8x8 transform in an SP slice");
        S.slice_tab[si].qs_c[0] = mb.QsC[0];          // interpret_mb.cc:799-801 (one value per slice)
        S.slice_tab[si].qs_c[1] = mb.QsC[1];
    }
    // the MB's storage position (mb_t::mb; MBAFF: row 2 pair_row + bottom, include/h264r.h)
    const int sidx = mb.mb.y * slice.active_sps->PicWidthInMbs + mb.mb.x;
    StagedMb& st = S.mbs[sidx];
    h264r_mb& r = st.rec;
    memset(&r, 0, sizeof(r));
    r.mb_type = mb.mb_type;
    r.flags = (mb.is_intra_block ? H264R_MBF_INTRA : 0) | (mb.transform_size_8x8_flag ? H264R_MBF_T8x8 : 0) |
              (mb.TransformBypassModeFlag ? H264R_MBF_BYPASS : 0) |
              (slice.header.MbaffFrameFlag && mb.mb_field_decoding_flag ? H264R_MBF_FIELD : 0);
    const int cbpl = mb.CodedBlockPatternLuma, cbpc = mb.CodedBlockPatternChroma;
    r.cbp = (uint8_t)(cbpl | cbpc << 4);
    r.qp_y = mb.QpY;
    r.qp_c[0] = mb.QpC[0]; r.qp_c[1] = mb.QpC[1];
    r.i16_mode = mb.Intra16x16PredMode;
    r.chroma_mode = mb.intra_chroma_pred_mode;
    r.cbp_blks = (uint16_t)(mb.cbp_blks[0] & 0xFFFF);
    r.slice = (uint16_t)si;
    for (int k = 0; k < 3; ++k) r.qp_scaled[k] = mb.qp_scaled[k];
    if (mb.mb_type == I_8x8)
        for (int b = 0; b < 4; ++b) r.ipred[b >> 1] |= (uint8_t)((mb.Intra8x8PredMode[b] & 15) << ((b & 1) * 4));
    else if (mb.mb_type == I_4x4)
        for (int b = 0; b < 16; ++b) r.ipred[b >> 1] |= (uint8_t)((mb.Intra4x4PredMode[b] & 15) << ((b & 1) * 4));
    else if (mb.TransformBypassModeFlag && !mb.is_intra_block) {
        // a lossless inter MB: the reference's bypass DPCM reads the mb_t slot's
        // Intra4x4PredMode / Intra8x8PredMode (transform.cc:993,1008), which the parser does
        // not reset for inter MBs -- pass on whatever they hold
        if (mb.transform_size_8x8_flag)
            for (int b = 0; b < 4; ++b) r.ipred[b >> 1] |= (uint8_t)((mb.Intra8x8PredMode[b] & 15) << ((b & 1) * 4));
        else
            for (int b = 0; b < 16; ++b) r.ipred[b >> 1] |= (uint8_t)((mb.Intra4x4PredMode[b] & 15) << ((b & 1) * 4));
    }

    // the level block (include/h264r.h layout) from the raw levels in cof
    std::vector<int16_t>& lv = st.levels;
    lv.clear();
    const int cfi = slice.active_sps->chroma_format_idc;
    const bool f422 = cfi == 2, f444 = cfi == 3, f400 = cfi == 0;
    const int MWc = f400 ? 0 : f444 ? 16 : 8, MHc = f400 ? 0 : cfi == 1 ? 8 : 16, nbc = f422 ? 8 : 4;   // MbWidthC, MbHeightC
    if (mb.mb_type == I_PCM) {
        lv.resize(128 + MWc * MHc);
        uint8_t* raw = reinterpret_cast<uint8_t*>(lv.data());
        for (int y = 0; y < 16; ++y) for (int x = 0; x < 16; ++x) raw[y * 16 + x] = (uint8_t)cof[0][y][x];
        for (int p = 0; p < 2; ++p)
            for (int y = 0; y < MHc; ++y)
                for (int x = 0; x < MWc; ++x) raw[256 + p * MWc * MHc + y * MWc + x] = (uint8_t)cof[1 + p][y][x];
    } else if (f444 || f400) {
        // three luma-like blocks, Y then Cb then Cr (4:0:0: the luma one): the coded 8x8 blocks,
        // then the I_16x16 DC
        for (int pl = 0; pl < (f400 ? 1 : 3); ++pl) {
            for (int b8 = 0; b8 < 4; ++b8) {
                if (!((cbpl >> b8) & 1)) continue;
                const int x8 = (b8 & 1) * 8, y8 = (b8 >> 1) * 8;
                if (!mb.transform_size_8x8_flag) {
                    for (int k = 0; k < 4; ++k)
                        for (int i = 0; i < 16; ++i)
                            lv.push_back((int16_t)cof[pl][y8 + (k >> 1) * 4 + i / 4][x8 + (k & 1) * 4 + i % 4]);
                    if (mb.mb_type == I_16x16)
                        for (int k = 0; k < 4; ++k) lv[lv.size() - 64 + k * 16] = 0;
                } else {
                    for (int i = 0; i < 64; ++i) lv.push_back((int16_t)cof[pl][y8 + i / 8][x8 + i % 8]);
                }
            }
            if (mb.mb_type == I_16x16)
                for (int i = 0; i < 16; ++i) lv.push_back((int16_t)cof[pl][(i / 4) * 4][(i % 4) * 4]);
        }
    } else if (f422) {
        // 4:2:2 (include/h264r.h): the luma part, then chroma AC (8 blocks per plane), then DC
        for (int b8 = 0; b8 < 4; ++b8) {
            if (!((cbpl >> b8) & 1)) continue;
            const int x8 = (b8 & 1) * 8, y8 = (b8 >> 1) * 8;
            if (!mb.transform_size_8x8_flag) {
                for (int k = 0; k < 4; ++k)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back((int16_t)cof[0][y8 + (k >> 1) * 4 + i / 4][x8 + (k & 1) * 4 + i % 4]);
                if (mb.mb_type == I_16x16)
                    for (int k = 0; k < 4; ++k) lv[lv.size() - 64 + k * 16] = 0;
            } else {
                for (int i = 0; i < 64; ++i) lv.push_back((int16_t)cof[0][y8 + i / 8][x8 + i % 8]);
            }
        }
        if (mb.mb_type == I_16x16)
            for (int i = 0; i < 16; ++i) lv.push_back((int16_t)cof[0][(i / 4) * 4][(i % 4) * 4]);
        if (cbpc == 2)
            for (int p = 1; p <= 2; ++p)
                for (int b = 0; b < nbc; ++b)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back(i == 0 ? 0 : (int16_t)cof[p][(b >> 1) * 4 + i / 4][(b & 1) * 4 + i % 4]);
        if (cbpc)
            for (int p = 1; p <= 2; ++p)
                for (int q = 0; q < nbc; ++q) lv.push_back((int16_t)cof[p][(q / 2) * 4][(q % 2) * 4]);
    } else {
        for (int b8 = 0; b8 < 4; ++b8) {
            if (!((cbpl >> b8) & 1)) continue;
            const int x8 = (b8 & 1) * 8, y8 = (b8 >> 1) * 8;
            if (!mb.transform_size_8x8_flag) {
                for (int k = 0; k < 4; ++k)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back((int16_t)cof[0][y8 + (k >> 1) * 4 + i / 4][x8 + (k & 1) * 4 + i % 4]);
                if (mb.mb_type == I_16x16)                    // the DC positions belong to the DC section
                    for (int k = 0; k < 4; ++k) lv[lv.size() - 64 + k * 16] = 0;
            } else {
                for (int i = 0; i < 64; ++i) lv.push_back((int16_t)cof[0][y8 + i / 8][x8 + i % 8]);
            }
        }
        if (cbpc == 2)
            for (int p = 1; p <= 2; ++p)
                for (int b = 0; b < 4; ++b)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back(i == 0 ? 0 : (int16_t)cof[p][(b >> 1) * 4 + i / 4][(b & 1) * 4 + i % 4]);
        if (mb.mb_type == I_16x16)
            for (int i = 0; i < 16; ++i) lv.push_back((int16_t)cof[0][(i / 4) * 4][(i % 4) * 4]);
        if (cbpc)
            for (int p = 1; p <= 2; ++p)
                for (int q = 0; q < 4; ++q) lv.push_back((int16_t)cof[p][(q / 2) * 4][(q % 2) * 4]);
    }
    // the MB's 16 motion entries per list (pic_motion_params, picture.h:66-71)
    for (int k = 0; k < 16; ++k) {
        const pic_motion_params& m = slice.dec_picture->mv_info[mb.mb.y * 4 + k / 4][mb.mb.x * 4 + k % 4];
        for (int l = 0; l < 2; ++l) {
            // a list is in use when it names a picture: P_Skip writes list 0 only, and list 1
            // keeps the zeroed ref_idx of a fresh mv_info (interpret_mv.cc:158-184) with a
            // NULL ref_pic -- which is what deblocking compares (deblock.cc:44-72)
            st.mv[l][k] = (uint32_t)(uint16_t)m.mv[l].mv_x | (uint32_t)(uint16_t)m.mv[l].mv_y << 16;
            st.ref[l][k] = m.ref_pic[l] ? (int8_t)m.ref_idx[l] : (int8_t)-1;
        }
    }
    S.seen[sidx] = 1;

    // coefficient-reset protocol (slice_data.cc:496-503): the same side effects as the
    // reference's reconstruction leaves behind
    if (f444) {                                                                          // decoder.cc:72-76
        slice.parser.is_reset_coeff = false;
        slice.parser.is_reset_coeff_cr = false;
    } else if (mb.mb_type != I_PCM) {
        if (mb.is_intra_block) {
            if (mb.mb_type == I_16x16 || cbpl || cbpc) slice.parser.is_reset_coeff = false;   // decoder.cc:196-197
            if (cbpc) slice.parser.is_reset_coeff_cr = false;                                // decoder.cc:205-206
        } else {
            if (cbpl || cbpc) slice.parser.is_reset_coeff = false;                           // decoder.cc:260-261
            if (cbpc) slice.parser.is_reset_coeff_cr = false;                                // transform.cc:1093-1094
        }
    }
}

void Decoder::deblock_filter(slice_t& slice)
{
    Shim& S = shim();
    storable_picture* pic = slice.dec_picture;
    if (S.pic != pic) check(H264R_ESTATE, "deblock_filter() of a picture that was not staged");
    const sps_t& sps = *slice.active_sps;
    const pps_t& pps = *slice.active_pps;
    const shr_t& shr = slice.header;
    const int W = sps.PicWidthInMbs, H = shr.PicHeightInMbs;        // a field: half the frame's rows
    const bool fld = shr.field_pic_flag;
    if (!S.have_quant) {
        h264r_quant q;
        check(h264r_quant_init_flat(&q), "h264r_quant_init_flat");
        S.quant = q;
    }
    h264r_pic p;
    memset(&p, 0, sizeof(p));
    p.constrained_intra_pred = pps.constrained_intra_pred_flag;
    p.num_slices = (int)S.slice_tab.size();
    p.poc = pic->poc;
    p.structure = !fld ? (shr.MbaffFrameFlag ? H264R_MBAFF_FRAME : H264R_FRAME)
                       : shr.bottom_field_flag ? H264R_BOTTOM_FIELD : H264R_TOP_FIELD;
    check(h264r_picture_begin(S.ctx, W, H, &p, S.slice_tab.data(), &S.quant), "h264r_picture_begin");
    for (int a = 0; a < W * H; ++a) {
        if (!S.seen[a]) check(H264R_ESTATE, "picture with missing macroblocks (concealment is CPU-only)");
        StagedMb& st = S.mbs[a];
        check(h264r_mb_submit(S.ctx, a, &st.rec, st.levels.empty() ? nullptr : st.levels.data(), (int)st.levels.size(),
                              &st.mv[0][0], &st.ref[0][0]), "h264r_mb_submit");
    }
    int keep = -1;
    const dpb_t* dpb = slice.p_Dpb;
    // an IDR picture empties the DPB (idr_memory_management, store_picture dpb.cc:888-891):
    // nothing resident before it can be referenced again
    if (pic->slice.idr_flag) S.slot_of.clear();
    if (pic->used_for_reference && fld && dpb && dpb->last_picture) {
        // the second field of a pair goes into its first field's slot: the pairing test of
        // store_picture (dpb.cc:903-912) -- the stored field of the opposite parity, the same
        // frame number, both reference fields
        const pic_t* fs = dpb->last_picture;
        const bool opposite = (pic->slice.structure == TOP_FIELD && fs->is_used == 2) ||
                              (pic->slice.structure == BOTTOM_FIELD && fs->is_used == 1);
        if ((int)fs->FrameNum == pic->PicNum && opposite && fs->is_orig_reference != 0)
            keep = decoded_slot(S, fs->is_used == 1 ? fs->top_field : fs->bottom_field);
    }
    if (pic->used_for_reference && keep < 0) {
        // a device slot no reference of the DPB holds: the frame stores of fs_ref / fs_ltref
        // (dpb.h:30-36) as they stand before this picture is stored (exit_picture ->
        // store_picture, picture.cc:253-269; its own marking can only free more), searched
        // round robin from the last slot given out.  The DPB holds <= 16 reference frames,
        // so one of the 32 slots is always free -- a long-term reference keeps its slot for
        // as long as it stays in the DPB.
        bool busy[H264R_MAX_SLOTS] = {};
        auto mark = [&](pic_t* fs) {
            if (!fs) return;
            for (const storable_picture* q : {fs->frame, fs->top_field, fs->bottom_field}) {
                int s = -1;
                if (q && q->slice.structure == FRAME) s = device_ref(S, q, false);
                else if (q) s = device_ref(S, q, true) & ~H264R_REF_BOTTOM;
                if (s >= 0) busy[s] = true;
            }
        };
        for (unsigned i = 0; dpb && i < dpb->ref_frames_in_buffer; ++i) mark(dpb->fs_ref[i]);
        for (unsigned i = 0; dpb && i < dpb->ltref_frames_in_buffer; ++i) mark(dpb->fs_ltref[i]);
        for (int k = 0; k < H264R_MAX_SLOTS && keep < 0; ++k)
            if (!busy[(S.next_slot + k) % H264R_MAX_SLOTS]) keep = (S.next_slot + k) % H264R_MAX_SLOTS;
        if (keep < 0) check(H264R_EUNSUPPORTED, "more than 32 reference frames resident");
        S.next_slot = (keep + 1) % H264R_MAX_SLOTS;
        for (auto it = S.slot_of.begin(); it != S.slot_of.end();)
            it = it->second.slot == keep ? S.slot_of.erase(it) : std::next(it);
    }
    const int MWc = S.ctx_cf == 0 ? 0 : S.ctx_cf == 3 ? 16 : 8;           // MbWidthC (4:0:0: no chroma planes)
    const int MHc = S.ctx_cf == 0 ? 0 : S.ctx_cf == 1 ? 8 : 16;           // MbHeightC
    S.y8.resize((size_t)W * H * 256);
    S.u8.resize((size_t)W * H * MWc * MHc);
    S.v8.resize((size_t)W * H * MWc * MHc);
    check(h264r_picture_end(S.ctx, S.y8.data(), S.u8.data(), S.v8.data(), keep), "h264r_picture_end");
    S.slot_of.erase(pic);
    if (keep >= 0) S.slot_of[pic] = Shim::Resident{keep, pic->slice.structure, pic->poc, pic->frame_num};
    for (int y = 0; y < H * 16; ++y)
        for (int x = 0; x < W * 16; ++x) pic->imgY[y][x] = S.y8[(size_t)y * W * 16 + x];
    for (int y = 0; y < H * MHc; ++y)
        for (int x = 0; x < W * MWc; ++x) {
            pic->imgUV[0][y][x] = S.u8[(size_t)y * W * MWc + x];
            pic->imgUV[1][y][x] = S.v8[(size_t)y * W * MWc + x];
        }
    S.pic = nullptr;
}

void Decoder::get_block_luma(storable_picture* curr_ref, int x_pos, int y_pos, int block_size_x, int block_size_y,
                             px_t block[16][16], int pl, mb_t& mb)
{
    this->inter_prediction->get_block_luma(curr_ref, x_pos, y_pos, block_size_x, block_size_y, block, pl, mb);
}

}
}
