// h264p.cc -- the repo's own CPU entropy / syntax stage.
//
// Annex-B stream -> NAL units -> SPS / PPS / slice headers -> CAVLC / CABAC macroblock layer ->
// per-picture staging -> the h264r reconstruction ABI (include/h264r.h), with the same
// records, levels, motion, slice tables, quantisation tables and DPB slots the reference
// parser + drop-in shim hand it (shim/decoder_h264r.cc).  Every function follows the
// reference behaviour it cites (R = luuvish/arrow-h264, H = R/src/codec/h264); where the
// reference keeps state the spec leaves undefined (mb_t fields not reset per MB,
// slice_data.cc:455-524) the parser keeps the same state, so its records are the shim's
// byte for byte (tests/test_parser.py compares them with the committed captures).
#include "h264p.h"

#include <algorithm>
#include <bitset>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "cabac_tables.h"
#include "cavlc_tables.h"
#include "h264r.h"

namespace h264p {
namespace {

struct Error {
    int status;
    std::string what;
};
[[noreturn]] void fail(int st, const std::string& what) { throw Error{st, what}; }
void require(bool ok, const char* what) { if (!ok) fail(H264R_EINVAL, what); }
void unsupported(bool bad, const char* what) { if (bad) fail(H264R_EUNSUPPORTED, what); }
void check(int st, const char* what) { if (st != H264R_OK) fail(st, std::string(what) + ": " + h264r_strerror(st)); }

template <typename T> T clip3(T lo, T hi, T v) { return v < lo ? lo : v > hi ? hi : v; }
int median(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }

// ------------------------------------------------------------------ bit reader
// RBSP of one NAL unit: emulation-prevention bytes removed (7.4.1), the rbsp_stop_one_bit
// located once for more_rbsp_data (bitstream.cc).
struct Bits {
    std::vector<uint8_t> buf;
    size_t pos = 0, nbits = 0, stop = 0;

    void load(const uint8_t* p, size_t n)
    {
        buf.clear();
        buf.reserve(n + 8);
        int zeros = 0;
        for (size_t i = 0; i < n; ++i) {
            if (zeros >= 2 && p[i] == 3) { zeros = 0; continue; }
            buf.push_back(p[i]);
            zeros = p[i] == 0 ? zeros + 1 : 0;
        }
        nbits = buf.size() * 8;
        stop = 0;
        for (size_t i = buf.size(); i-- > 0;)
            if (buf[i]) { stop = i * 8 + 7 - __builtin_ctz(buf[i]); break; }
        buf.insert(buf.end(), 8, 0);
        pos = 0;
    }
    // the n (1..32) bits at bit position p, zeros past the end (one big-endian 8-byte load
    // inside the buffer, which ends in 8 zero bytes)
    uint32_t peek_at(size_t p, int n) const
    {
        const size_t b = p >> 3;
        uint64_t w = 0;
        if (b + 8 <= buf.size()) {
            memcpy(&w, &buf[b], 8);
            w = __builtin_bswap64(w);
        } else {
            for (size_t k = 0; k < 8; ++k) w = w << 8 | (b + k < buf.size() ? buf[b + k] : 0);
        }
        return (uint32_t)((w << (p & 7)) >> (64 - n));
    }
    uint32_t peek(int n) const { return peek_at(pos, n); }
    void skip(int n)
    {
        pos += n;
        if (pos > nbits) fail(H264R_EINVAL, "bitstream: read past the end of a NAL unit");
    }
    uint32_t bit()
    {
        if (pos >= nbits) fail(H264R_EINVAL, "bitstream: read past the end of a NAL unit");
        const uint32_t v = (buf[pos >> 3] >> (7 - (pos & 7))) & 1;
        ++pos;
        return v;
    }
    uint32_t u(int n)
    {
        if (n == 0) return 0;
        if (pos + n > nbits) fail(H264R_EINVAL, "bitstream: read past the end of a NAL unit");
        const uint32_t v = peek(n);
        pos += n;
        return v;
    }
    uint32_t ue()
    {
        const uint32_t w = peek_at(pos, 32);
        if (!w) fail(H264R_EINVAL, "bitstream: ue(v) longer than 32 bits");
        const int lz = __builtin_clz(w);                // the leading zeros, then the 1
        skip(lz + 1);
        return lz ? (uint32_t)((1ull << lz) - 1 + u(lz)) : 0;
    }
    int32_t se()
    {
        const uint32_t k = ue();
        return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
    }
    // ue(v) / se(v) of a syntax element with a range: out of it the stream is malformed (the
    // value never reaches an int field, where 2^31 and more would turn negative)
    int ue_max(uint32_t max, const char* what)
    {
        const uint32_t v = ue();
        require(v <= max, what);
        return (int)v;
    }
    int se_in(int lo, int hi, const char* what)
    {
        const int32_t v = se();
        require(v >= lo && v <= hi, what);
        return v;
    }
    bool aligned() const { return (pos & 7) == 0; }
    bool more_rbsp_data() const { return pos < stop; }
};

// A VLC table as a prefix lookup over its longest codeword: value | length << 8 of the
// codeword the next `bits` bits start with (length 0: no codeword).  Sized per table (total_zeros
// 9 bits, run_before 11, coeff_token up to 16), so the tables the residual reads stay in cache.
struct Vlc {
    int bits = 1;
    std::vector<uint16_t> e;
    template <typename E, typename F>
    void build(const E* c, int n, F value)
    {
        bits = 1;
        for (int i = 0; i < n; ++i) bits = std::max(bits, (int)c[i].len);
        e.assign((size_t)1 << bits, 0);
        for (int i = 0; i < n; ++i) {
            const int l = c[i].len, lo = c[i].code << (bits - l), hi = lo + (1 << (bits - l));
            for (int k = lo; k < hi; ++k) e[k] = (uint16_t)(value(c[i]) | l << 8);
        }
    }
    int read(Bits& b, const char* what) const
    {
        const uint16_t v = e[b.peek(bits)];
        if (!(v >> 8)) fail(H264R_EINVAL, std::string("bitstream: no ") + what + " codeword");
        b.skip(v >> 8);
        return v & 255;
    }
};

struct Tables {
    Vlc coeff_token[5];   // nC classes 0, 2, 4, -1, -2: value = TotalCoeff << 2 | TrailingOnes
    Vlc total_zeros[3][16];
    Vlc run_before[8];
    Tables()
    {
        auto ct = [](const CoeffTokenCode& e) { return e.total_coeff << 2 | e.trailing_ones; };
        coeff_token[0].build(CT_NC0, sizeof(CT_NC0) / sizeof(CT_NC0[0]), ct);
        coeff_token[1].build(CT_NC2, sizeof(CT_NC2) / sizeof(CT_NC2[0]), ct);
        coeff_token[2].build(CT_NC4, sizeof(CT_NC4) / sizeof(CT_NC4[0]), ct);
        coeff_token[3].build(CT_NCM1, sizeof(CT_NCM1) / sizeof(CT_NCM1[0]), ct);
        coeff_token[4].build(CT_NCM2, sizeof(CT_NCM2) / sizeof(CT_NCM2[0]), ct);
        auto v = [](const VlcCode& e) { return e.value; };
        for (int tc = 1; tc < (int)sizeof(TZ_0_N); ++tc) total_zeros[0][tc].build(TZ_0[tc], TZ_0_N[tc], v);
        for (int tc = 1; tc < (int)sizeof(TZ_1_N); ++tc) total_zeros[1][tc].build(TZ_1[tc], TZ_1_N[tc], v);
        for (int tc = 1; tc < (int)sizeof(TZ_2_N); ++tc) total_zeros[2][tc].build(TZ_2[tc], TZ_2_N[tc], v);
        for (int z = 1; z < 8; ++z) run_before[z].build(RB[z], RB_N[z], v);
    }
};
const Tables& tables()
{
    static const Tables t;
    return t;
}

// ------------------------------------------------------------------ CABAC engine
// cabac_engine_t (interpret.cc:308-432): 9-bit codIOffset read bit by bit from the RBSP, so
// the bit position after a terminating bin is exactly where the spec puts it (I_PCM samples
// and the slice end follow it); the contexts in the reference's layout (cabac_tables.h).
struct Cabac {
    Bits* b = nullptr;
    uint32_t range = 510;
    // codIOffset with k look-ahead bits below it: value = codIOffset << k | the next k bits of
    // the RBSP (loaded up to bit lpos), so RenormD only lowers k and the RBSP is read 32 bits
    // at a time; the exact bit position (lpos - k) is handed back to the RBSP where the spec
    // reads raw bits after a terminating bin (I_PCM samples)
    uint64_t value = 0;
    int k = 0;
    size_t lpos = 0;
    uint8_t st[CABAC_CONTEXTS];                        // pStateIdx << 1 | valMPS

    struct Trans {
        uint8_t mps[128], lps[128];
        Trans()
        {
            for (int s = 0; s < 64; ++s)
                for (int m = 0; m < 2; ++m) {
                    mps[s << 1 | m] = (uint8_t)(TRANS_MPS[s] << 1 | m);
                    lps[s << 1 | m] = (uint8_t)(TRANS_LPS[s] << 1 | (s == 0 ? 1 - m : m));
                }
        }
    };
    static const Trans& trans()
    {
        static const Trans t;
        return t;
    }

    // cabac_contexts_t::init (bitstream_cabac.cc:1215-1264): kind 0 = I, 1..3 = P idc, 4..6 = B idc
    void init_contexts(int kind, int qp)
    {
        qp = clip3(0, 51, qp);
        for (int i = 0; i < CABAC_CONTEXTS; ++i) {
            const int pre = clip3(1, 126, ((CABAC_MN[kind][i][0] * qp) >> 4) + CABAC_MN[kind][i][1]);
            st[i] = pre <= 63 ? (uint8_t)((63 - pre) << 1) : (uint8_t)((pre - 64) << 1 | 1);
        }
    }
    void refill()
    {
        value = value << 32 | b->peek_at(lpos, 32);
        lpos += 32;
        k += 32;
    }
    void init_engine(Bits& bits)                       // cabac_engine_t::init: byte-align, 9 bits
    {
        b = &bits;
        while (!b->aligned()) b->u(1);
        range = 510;
        value = b->u(9);
        lpos = b->pos;
        k = 0;
        refill();
    }
    int dec(int ctx)
    {
        const int s = st[ctx];
        const uint32_t lps = RANGE_LPS[s >> 1][(range >> 6) & 3];
        range -= lps;
        const uint64_t r = (uint64_t)range << k;
        int bin;
        if (value < r) {
            bin = s & 1;
            st[ctx] = trans().mps[s];
        } else {
            bin = !(s & 1);
            value -= r;
            range = lps;
            st[ctx] = trans().lps[s];
        }
        renorm();
        return bin;
    }
    void renorm()                                      // RenormD: range back to 9 bits at once
    {
        if (range < 256) {
            const int sh = __builtin_clz(range) - 23;
            range <<= sh;
            k -= sh;
            if (k < 16) refill();
        }
    }
    int bypass()
    {
        --k;
        const uint64_t r = (uint64_t)range << k;
        int bin = 0;
        if (value >= r) {
            value -= r;
            bin = 1;
        }
        if (k < 16) refill();
        return bin;
    }
    void check_end() const
    {
        if (lpos - k > b->nbits) fail(H264R_EINVAL, "bitstream: read past the end of a NAL unit");
    }
    int term()
    {
        range -= 2;
        check_end();
        if (value >= (uint64_t)range << k) {
            b->pos = lpos - k;                         // the RBSP continues here (I_PCM samples)
            return 1;
        }
        renorm();
        return 0;
    }
    // u / tu / ueg / fl binarisations (interpret.cc:383-432); inc[k] = ctxIdxInc of bin k
    // (the last entry for every later bin)
    int unary(int ctx, const int* inc, int ninc)
    {
        int n = 0;
        while (dec(ctx + inc[std::min(n, ninc - 1)])) {
            if (++n > 4096) fail(H264R_EINVAL, "CABAC: unary code too long");
        }
        return n;
    }
    int tu(int ctx, const int* inc, int ninc, int cmax)
    {
        int n = 0;
        while (n < cmax && dec(ctx + inc[std::min(n, ninc - 1)])) ++n;
        return n;
    }
    int ueg(int ctx, const int* inc, int ninc, int cmax, int k, bool sign)
    {
        int v = tu(ctx, inc, ninc, cmax);
        if (v == cmax) {
            while (bypass()) {
                v += 1 << k++;
                if (k > 24) fail(H264R_EINVAL, "CABAC: exp-Golomb suffix too long");
            }
            while (k--) v += bypass() << k;
        }
        if (sign && v && bypass()) v = -v;
        return v;
    }
};

// zig-zag scans (frame): raster index of scan position k (Tables 8-12 / 8-13)
const uint8_t ZZ4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
const uint8_t ZZ8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Table 8-15 (interpret_mb.cc:777-782)
const uint8_t QP_SCALE_CR[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                                 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

// Flat / default scaling lists (Tables 7-3, 7-4), raster order
const int32_t FLAT16[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
                            16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
                            16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16};
const int32_t DEF4_INTRA[16] = {6, 13, 20, 28, 13, 20, 28, 32, 20, 28, 32, 37, 28, 32, 37, 42};
const int32_t DEF4_INTER[16] = {10, 14, 20, 24, 14, 20, 24, 27, 20, 24, 27, 30, 24, 27, 30, 34};
const int32_t DEF8_INTRA[64] = {6,  10, 13, 16, 18, 23, 25, 27, 10, 11, 16, 18, 23, 25, 27, 29, 13, 16, 18, 23, 25, 27,
                                29, 31, 16, 18, 23, 25, 27, 29, 31, 33, 18, 23, 25, 27, 29, 31, 33, 36, 23, 25, 27, 29,
                                31, 33, 36, 38, 25, 27, 29, 31, 33, 36, 38, 40, 27, 29, 31, 33, 36, 38, 40, 42};
const int32_t DEF8_INTER[64] = {9,  13, 15, 17, 19, 21, 22, 24, 13, 13, 17, 19, 21, 22, 24, 25, 15, 17, 19, 21, 22, 24,
                                25, 27, 17, 19, 21, 22, 24, 25, 27, 28, 19, 21, 22, 24, 25, 27, 28, 30, 21, 22, 24, 25,
                                27, 28, 30, 32, 22, 24, 25, 27, 28, 30, 32, 33, 24, 25, 27, 28, 30, 32, 33, 35};

// ------------------------------------------------------------------ parameter sets
struct ScalingLists {
    bool matrix_present = false;
    bool list_present[12] = {};
    int32_t sl4[6][16] = {};
    int32_t sl8[6][64] = {};
    bool def4[6] = {}, def8[6] = {};
};

// scaling_list() (interpret_rbsp.cc:272-287): delta_scale kept as int8, values at raster
// positions through the zig-zag scan
void scaling_list(Bits& b, int32_t* list, int size, bool& use_default)
{
    int last = 8, next = 8;
    for (int j = 0; j < size; ++j) {
        const int scanj = size == 16 ? ZZ4[j] : ZZ8[j];
        if (next != 0) {
            const int8_t delta = (int8_t)b.se();
            next = (last + delta + 256) % 256;
            use_default = scanj == 0 && next == 0;
        }
        list[scanj] = next == 0 ? last : next;
        last = list[scanj];
    }
}

void scaling_matrix(Bits& b, ScalingLists& s, int n)
{
    for (int i = 0; i < n; ++i) {
        s.list_present[i] = b.u(1);
        if (s.list_present[i]) {
            if (i < 6) scaling_list(b, s.sl4[i], 16, s.def4[i]);
            else scaling_list(b, s.sl8[i - 6], 64, s.def8[i - 6]);
        }
    }
}

struct Sps {
    bool valid = false;
    int profile = 0, chroma_format_idc = 1, bit_depth_y = 8, bit_depth_c = 8;
    bool bypass = false;
    ScalingLists sc;
    int log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4;
    int max_num_ref_frames = 0;
    bool gaps = false;
    int W = 0, H = 0;
    bool frame_mbs_only = true, mbaff = false, direct_8x8_inference = false, separate_planes = false;
    int crop[4] = {0, 0, 0, 0};   // left, right, top, bottom (frame_crop_*_offset)
};

struct Pps {
    bool valid = false;
    int sps_id = 0;
    bool cabac = false, bottom_field_poc = false;
    int num_slice_groups = 1;
    int nref_default[2] = {1, 1};
    bool weighted_pred = false;
    int weighted_bipred_idc = 0;
    int init_qp = 26, init_qs = 26;
    int cqp_offset[2] = {0, 0};
    bool deblocking_control = false, cip = false, redundant_pic_cnt = false;
    bool transform_8x8 = false;
    ScalingLists sc;
};

// seq_parameter_set_rbsp (7.3.2.1.1; interpret_rbsp.cc): the set and its id
int parse_sps(Bits& b, Sps& s)
{
    s = Sps();
    s.profile = b.u(8);
    b.u(16);                                  // constraint flags, level_idc
    const int id = b.ue_max(31, "SPS: seq_parameter_set_id");
    if (s.profile == 100 || s.profile == 110 || s.profile == 122 || s.profile == 244 || s.profile == 44 ||
        s.profile == 83 || s.profile == 86 || s.profile == 118 || s.profile == 128 || s.profile == 138 ||
        s.profile == 139 || s.profile == 134 || s.profile == 135) {
        s.chroma_format_idc = b.ue_max(3, "SPS: chroma_format_idc");
        if (s.chroma_format_idc == 3) s.separate_planes = b.u(1);   // separate_colour_plane_flag
        s.bit_depth_y = 8 + b.ue_max(6, "SPS: bit_depth_luma_minus8");
        s.bit_depth_c = 8 + b.ue_max(6, "SPS: bit_depth_chroma_minus8");
        s.bypass = b.u(1);
        s.sc.matrix_present = b.u(1);
        if (s.sc.matrix_present) scaling_matrix(b, s.sc, s.chroma_format_idc != 3 ? 8 : 12);
    }
    // the reference asserts log2_max_frame_num_minus4 <= 12 (interpret_rbsp.cc); the same range
    // bounds log2_max_pic_order_cnt_lsb_minus4 (7.4.2.1.1)
    s.log2_max_frame_num = b.ue_max(12, "SPS: log2_max_frame_num_minus4") + 4;
    s.poc_type = b.ue_max(2, "SPS: pic_order_cnt_type");
    if (s.poc_type == 0) s.log2_max_poc_lsb = b.ue_max(12, "SPS: log2_max_pic_order_cnt_lsb_minus4") + 4;
    else if (s.poc_type == 1) {
        b.u(1); b.se(); b.se();
        const int n = b.ue_max(255, "SPS: num_ref_frames_in_pic_order_cnt_cycle");
        for (int i = 0; i < n; ++i) b.se();
    }
    s.max_num_ref_frames = b.ue_max(16, "SPS: max_num_ref_frames");
    s.gaps = b.u(1);
    // picture sizes beyond the library's (1024 x 1024 MBs, include/h264r.h) are refused here,
    // before any buffer is sized from them
    s.W = b.ue_max(1023, "SPS: pic_width_in_mbs_minus1") + 1;
    const int map_h = b.ue_max(1023, "SPS: pic_height_in_map_units_minus1") + 1;
    s.frame_mbs_only = b.u(1);
    if (!s.frame_mbs_only) s.mbaff = b.u(1);
    s.H = map_h * (2 - s.frame_mbs_only);
    s.direct_8x8_inference = b.u(1);
    if (b.u(1))
        for (int k = 0; k < 4; ++k) s.crop[k] = b.ue_max(8 * 1024, "SPS: frame_crop offset");
    require(2 * (s.crop[0] + s.crop[1]) < 16 * s.W && 2 * (s.crop[2] + s.crop[3]) < 16 * s.H, "SPS: cropping window empty");
    // vui_parameters: nothing the path reads
    s.valid = true;
    return id;
}

// pic_parameter_set_rbsp (7.3.2.2): the set and its id
int parse_pps(Bits& b, Pps& p, const Sps* spss)
{
    p = Pps();
    const int id = b.ue_max(255, "PPS: pic_parameter_set_id");
    p.sps_id = b.ue_max(31, "PPS: seq_parameter_set_id");
    require(spss[p.sps_id].valid, "PPS: seq_parameter_set_id of no SPS");
    p.cabac = b.u(1);
    p.bottom_field_poc = b.u(1);
    p.num_slice_groups = b.ue_max(7, "PPS: num_slice_groups_minus1") + 1;
    unsupported(p.num_slice_groups > 1, "slice groups (FMO)");
    p.nref_default[0] = b.ue_max(31, "PPS: num_ref_idx_l0_default_active_minus1") + 1;
    p.nref_default[1] = b.ue_max(31, "PPS: num_ref_idx_l1_default_active_minus1") + 1;
    p.weighted_pred = b.u(1);
    p.weighted_bipred_idc = b.u(2);
    require(p.weighted_bipred_idc <= 2, "PPS: weighted_bipred_idc");
    p.init_qp = 26 + b.se_in(-26, 25, "PPS: pic_init_qp_minus26");
    p.init_qs = 26 + b.se_in(-26, 25, "PPS: pic_init_qs_minus26");
    p.cqp_offset[0] = b.se_in(-12, 12, "PPS: chroma_qp_index_offset");
    p.deblocking_control = b.u(1);
    p.cip = b.u(1);
    p.redundant_pic_cnt = b.u(1);
    p.cqp_offset[1] = p.cqp_offset[0];
    if (b.more_rbsp_data()) {
        p.transform_8x8 = b.u(1);
        p.sc.matrix_present = b.u(1);
        if (p.sc.matrix_present)
            scaling_matrix(b, p.sc, 6 + (spss[p.sps_id].chroma_format_idc != 3 ? 2 : 6) * p.transform_8x8);
        p.cqp_offset[1] = b.se_in(-12, 12, "PPS: second_chroma_qp_index_offset");
    }
    p.valid = true;
    return id;
}

// Transform::init fall-back rules A / B (transform.cc:173-257), as restated by the shim
// (shim/decoder_h264r.cc assign_quant_params): qmatrix[12] -> h264r_quant
h264r_quant quant_tables(const Sps& sps, const Pps& pps)
{
    const int32_t* qm[12];
    if (!pps.sc.matrix_present && !sps.sc.matrix_present) {
        for (int i = 0; i < 12; ++i) qm[i] = FLAT16;
    } else {
        for (int i = 0; i < 12; ++i) qm[i] = i < 6 ? DEF4_INTRA : DEF8_INTRA;
        const int n = sps.chroma_format_idc != 3 ? 8 : 12;
        auto apply = [&](const ScalingLists& s, bool fallback_a) {
            for (int i = 0; i < n; ++i) {
                if (i < 6) {
                    if (!s.list_present[i]) {
                        if (fallback_a) qm[i] = i == 0 ? DEF4_INTRA : i == 3 ? DEF4_INTER : qm[i - 1];
                        else if (i == 0) { if (!sps.sc.matrix_present) qm[i] = DEF4_INTRA; }
                        else if (i == 3) { if (!sps.sc.matrix_present) qm[i] = DEF4_INTER; }
                        else qm[i] = qm[i - 1];
                    } else
                        qm[i] = s.def4[i] ? (i < 3 ? DEF4_INTRA : DEF4_INTER) : s.sl4[i];
                } else {
                    if (!s.list_present[i]) {
                        if (fallback_a) qm[i] = i == 6 ? DEF8_INTRA : i == 7 ? DEF8_INTER : qm[i - 2];
                        else if (i == 6) { if (!sps.sc.matrix_present) qm[i] = DEF8_INTRA; }
                        else if (i == 7) { if (!sps.sc.matrix_present) qm[i] = DEF8_INTER; }
                        else qm[i] = qm[i - 2];
                    } else
                        qm[i] = s.def8[i - 6] ? ((i & 1) == 0 ? DEF8_INTRA : DEF8_INTER) : s.sl8[i - 6];
                }
            }
        };
        if (sps.sc.matrix_present) apply(sps.sc, true);
        if (pps.sc.matrix_present) apply(pps.sc, false);
        if (n == 8)
            for (int i = 8; i < 12; ++i) qm[i] = qm[i - 2];
    }
    h264r_quant q;
    check(h264r_quant_init_lists(&q, qm), "h264r_quant_init_lists");
    return q;
}

// ------------------------------------------------------------------ pictures / DPB
struct Motion {
    int W4 = 0, H4 = 0;
    std::vector<int8_t> ref_idx[2];     // as the parser writes mv_info.ref_idx (-1 = none)
    std::vector<int16_t> mvx[2], mvy[2];
    std::vector<int32_t> ref_pic[2];    // picture id of mv_info.ref_pic (-1 = NULL)
    void init(int W, int H)
    {
        W4 = 4 * W; H4 = 4 * H;
        for (int l = 0; l < 2; ++l) {
            // a fresh mv_info: zeros, no picture (P_Skip writes list 0 only, interpret_mv.cc:177-184)
            ref_idx[l].assign((size_t)W4 * H4, 0);
            mvx[l].assign((size_t)W4 * H4, 0);
            mvy[l].assign((size_t)W4 * H4, 0);
            ref_pic[l].assign((size_t)W4 * H4, -1);
        }
    }
    size_t at(int x4, int y4) const { return (size_t)y4 * W4 + x4; }
};

// A frame store (the reference's pic_t, dpb.h): a frame, or the field pair a frame was coded
// as (PAFF).  Its field views (`view`, created on demand) are the list entries of field
// pictures (dpb_split_field picture.cc:408-470 without the copy: on the device a field is every
// second row of the frame store's slot, include/h264r.h H264R_REF_BOTTOM).
struct Picture {
    int id = 0;
    int poc = 0, frame_num = 0, frame_num_wrap = 0;
    bool idr = false;
    bool ref = false;              // used for (short- or long-term) reference (a field pair: either field)
    bool long_term = false;
    int lt_idx = 0;
    int slot = -1;                 // device DPB slot (reference pictures)
    std::shared_ptr<Motion> mot;
    // field coding (PAFF)
    bool fields = false;           // coded as field pictures
    bool has[2] = {true, true};    // top / bottom present (is_used bits)
    bool ref_f[2] = {false, false};   // top / bottom used for reference
    int poc_f[2] = {0, 0};         // TopFieldOrderCnt / BottomFieldOrderCnt
    std::shared_ptr<Motion> mot_f[2];  // a field pair's top / bottom field motion
    Picture* parent = nullptr;     // a field view: its frame store
    int parity = 0;                // a field view: 0 top, 1 bottom
    std::unique_ptr<Picture> view[2];
    // the field view of parity k (POC, long-term state and identity of that field)
    Picture* field(int k, int& next_id)
    {
        if (!view[k]) {
            view[k] = std::make_unique<Picture>();
            view[k]->id = next_id++;
            view[k]->parent = this;
            view[k]->parity = k;
        }
        Picture* v = view[k].get();
        v->poc = poc_f[k];
        v->frame_num = frame_num;
        v->long_term = long_term;
        v->lt_idx = lt_idx;
        v->ref = ref_f[k];
        return v;
    }
};

struct Output {
    int period, poc;
    int W, H, crop[4];              // its SPS's, at the time it was decoded (a later SPS may differ)
    std::vector<uint8_t> y, u, v;
    int cf = 1;                     // chroma_format_idc (4:2:2: chroma planes of 8 x 16 per MB)
};

// ------------------------------------------------------------------ slice header
struct Mmco {
    int op, a, b;
};
struct ListMod {
    int idc, val;
};
struct SliceHeader {
    int nal_ref_idc = 0, nal_type = 0;
    bool idr = false;
    bool field = false, bottom = false;   // field_pic_flag, bottom_field_flag (PAFF)
    int first_mb = 0, slice_type = 0, pps_id = 0;
    int frame_num = 0, idr_pic_id = 0, poc_lsb = 0, delta_poc_bottom = 0;
    bool direct_spatial = false;
    int nref[2] = {0, 0};
    bool mod_flag[2] = {false, false};
    std::vector<ListMod> mods[2];
    int luma_log2_wd = 5, chroma_log2_wd = 5;
    int weight[2][32][3] = {}, offset[2][32][3] = {};
    bool no_output_of_prior_pics = false, long_term_reference = false, adaptive = false;
    std::vector<Mmco> mmco;
    int cabac_init_idc = 0;
    int qp = 26, qs = 0;
    bool sp_switch = false;
    int deblock_idc = 0, offset_a = 0, offset_b = 0;
};

// ------------------------------------------------------------------ per-MB state
// The mb_t fields the parser reads back from neighbours or that leave the reference's
// mb_data array unreset between pictures (slice_data.cc:455-524: intra modes, I16 mode).
struct MbState {
    int slice_nr = -1;
    bool intra = false;
    uint8_t mb_type = 0;
    bool t8 = false;
    uint8_t i4[16] = {}, i8[4] = {}, i16 = 0;
    uint8_t nz[3][4][4] = {};             // CAVLC TotalCoeff per 4x4 block (nz_coeff)
    uint8_t sub_type[4] = {}, sub_pred[4] = {};
    // read by the CABAC context selection (neighbour.cc:415-764)
    bool skip = false;
    bool fld = false;                     // mb_field_decoding_flag (MBAFF frames)
    uint8_t cbpl = 0, cbpc = 0, cmode = 0;
    uint64_t cbp_bits = 0;                // coded_block_flag bits (update_coded_block_flag)
    int16_t mvd[2][16][2] = {};           // mvd_l0 / mvd_l1 per 4x4 block (raster)
};

struct StagedMb {
    h264r_mb rec;
    std::vector<int16_t> levels;
    uint32_t mv[2][16];
    int8_t ref[2][16];
};

class Decoder;

// One slice's macroblock layer (interpret_mb.cc, interpret_mv.cc, interpret_residual.cc)
struct SliceCtx {
    Decoder& D;
    const Sps& sps;
    const Pps& pps;
    const SliceHeader& sh;
    int slice_nr;
    Bits& b;
    int W, H;                   // the picture's MBs (a field picture: FrameHeightInMbs / 2 rows)
    int cf, mwc, mhc;           // chroma_format_idc (1, 2, 3), MbWidthC (8, 16) and MbHeightC (8, 16)
    const uint8_t* zz4;         // inverse scans: frame zig-zag, or the field scans of a field picture
    const uint8_t* zz8;
    int qp;                     // slice.parser.QpY
    int skip_run = -1;
    bool mbaff;                 // MbaffFrameFlag: MB pairs, addr an MB address, the state at its storage index
    int run_now = 0;            // mb_skip_run as read for the current MB (before its decrement)
    // MBAFF CABAC: a skipped top MB reads its bottom MB's mb_skip_flag (and, if coded, the pair's
    // mb_field_decoding_flag) ahead (interpret_mb.cc:210-231 prescan_*)
    bool pre_skip_read = false, pre_skip = false, pre_fld_read = false, pre_fld = false;
    int cabac_field_flag();
    Cabac* cab = nullptr;       // CABAC slices (entropy_coding_mode_flag)
    int last_dquant = 0;
    // the current MB (addr its MB address; MBAFF: stored at row mby = 2 pair_row + addr % 2, include/h264r.h)
    int addr = 0, si = 0, mbx = 0, mby = 0;
    MbState* cur = nullptr;
    int cbpl = 0, cbpc = 0, qpy = 0, qpc[2] = {0, 0}, qsc[2] = {0, 0}, qp_scaled[3] = {0, 0, 0};
    bool bypass = false, skip = false, allrefzero = false, no_sub_lt8 = true;
    uint8_t chroma_mode = 0;
    uint16_t cbp_blks = 0;
    int32_t cof[3][16][16];

    Picture* const (*list_)[33];  // RefPicList of this slice (the slices of a picture may run in parallel)
    const int* list_n_;
    int end_mb;                   // the next slice's first MB (a slice running into it is malformed)

    SliceCtx(Decoder& d, const Sps& s, const Pps& p, const SliceHeader& h, int nr, Bits& bits,
             Picture* const (*lists)[33], const int* list_n, int end);
    void run();
    void macroblock();
    MbState* nb_mb(bool chroma, int xN, int yN, int& ax, int& ay);
    void update_qp(int q);
    void intra_pred_modes();
    uint8_t pred_mode(int bx, int by, bool n8);
    void inter_pred();
    void reset_motion();
    void skip_p();
    void neighbour_mv(int list, int i, int j, int w, int h, bool avail[3], int ref[3], int mv[3][2]);
    void predict_mv(const bool avail[3], const int ref[3], const int mv[3][2], int refidx, int i, int j, int w, int h,
                    int out[2]);
    void direct_spatial();
    void direct_temporal();
    const Motion& colocated(int i4, int j4, size_t& e);
    void residual();
    int nnz_pred(int pl, int i, int j);
    int block_cavlc(int pl, bool chroma, bool ac, int blk, int start, int max_coeff, int32_t* coeff_pos_level,
                    int* npos);
    // CABAC syntax elements (interpret_se.cc, contexts neighbour.cc:415-764)
    MbState* nb_cur(int dx, int dy);
    int cabac_mb_type(bool I, bool B);
    int cabac_sub_mb_type(bool B);
    int cabac_cbp();
    int cabac_ref_idx(int list, int x4, int y4);
    int cabac_mvd(int list, int x4, int y4, int comp);
    int cbf_inc(int pl, bool chroma, bool ac, int blk);
    int block_cabac(int cat, int pl, bool chroma, bool ac, int blk, int start, int max_coeff, int32_t* out, int* nout);
    int block(int cat, int pl, bool chroma, bool ac, int blk, int start, int max_coeff, int32_t* out, int* nout)
    {
        return cab ? block_cabac(cat, pl, chroma, ac, blk, start, max_coeff, out, nout)
                   : block_cavlc(pl, chroma, ac, blk, start, max_coeff, out, nout);
    }
    void stage();
    bool read_t8();
    void set_cbp_state();
};

class Decoder {
public:
    explicit Decoder(int device) : device_(device) {}
    ~Decoder() { if (ctx_) h264r_destroy(ctx_); }
    int decode(const uint8_t* data, size_t size, h264p_output_fn out, void* user);
    std::string err;

    // state the slice layer reads
    Sps sps_[32];
    Pps pps_[256];
    std::vector<uint8_t> sps_raw_[32], pps_raw_[256];   // RBSP bytes of each stored set (repeats are no-ops)
    std::bitset<256> pps_used_;                       // PPS ids the open picture's slices refer to
    std::vector<MbState> mbs_;
    std::vector<StagedMb> staged_;
    std::vector<uint8_t> seen_;
    std::shared_ptr<Motion> mot_;             // current picture's motion
    Picture* list_[2][33] = {};                // RefPicList (frames)
    int list_n_[2] = {0, 0};
    std::vector<std::unique_ptr<Picture>> dpb_;  // reference pictures (+ the current one while decoding)
    Picture* cur_ = nullptr;
    int cur_poc_ = 0;                          // the current picture's POC (a field: its own)
    int pic_h_ = 0;                            // its height in MBs (a field: half the frame's)
    Picture* last_field_ = nullptr;            // a frame store holding one decoded field (dpb last_picture)
    std::vector<h264r_slice> slice_tab_;
    h264r_quant quant_;
    bool have_quant_ = false;
    // the picture's slices, parsed when the picture ends: on several threads when it has
    // several (slices never read each other's syntax: every neighbour across a slice edge is
    // "not available"), H264P_THREADS (default: up to 8) threads
    struct PendingSlice {
        SliceHeader h;
        Bits b;
        int nr;
        const Sps* sps;
        const Pps* pps;
        Picture* list[2][33];
        int list_n[2];
    };
    std::vector<std::unique_ptr<PendingSlice>> pslices_;
    void run_slices();

private:
    int device_;
    h264r_ctx* ctx_ = nullptr;
    int ctx_w_ = 0, ctx_h_ = 0, ctx_cf_ = 0, mbs_w_ = 0, mbs_h_ = 0;
    int next_id_ = 0, next_slot_ = 0;
    const Sps* psps_ = nullptr;
    const Pps* ppps_ = nullptr;
    SliceHeader first_;                        // header of the current picture's first slice
    bool in_picture_ = false;
    // POC state (8.2.1)
    int prev_poc_msb_ = 0, prev_poc_lsb_ = 0, prev_frame_num_ = 0, prev_frame_num_offset_ = 0;
    int max_lt_idx_ = -1;                      // MaxLongTermFrameIdx (-1: no long-term frame indices)
    int period_ = -1;
    int inflight_par_ = -1;                    // the picture on the GPU is a field of parity 0 / 1 (-1: frame)
    int out_of_first_ = -1;                    // pending_ entry of the open field pair's frame
    std::vector<uint8_t> fy_, fu_, fv_;        // a field's planes between the GPU and its frame's output
    std::vector<Output> pending_;
    h264p_output_fn out_ = nullptr;
    void* user_ = nullptr;
    int stop_ = 0;
    int inflight_ = -1;                        // pending_ entry whose planes are still on the GPU
    bool sync_ = getenv("H264P_SYNC") != nullptr;   // A/B switch: h264r_picture_end per picture

    void nal(const uint8_t* p, size_t n);
    void slice(Bits& b, int nal_ref_idc, int nal_type);
    void parse_slice_header(Bits& b, SliceHeader& h);
    void begin_picture(const SliceHeader& h);
    void finish_picture();
    void init_lists(const SliceHeader& h);
    void init_field_lists(const SliceHeader& h);
    void modify_list(const SliceHeader& h, int l);
    h264r_slice slice_record(const SliceHeader& h);
    void mark_picture();
    void flush_output();
    void collect();
};

// ------------------------------------------------------------------ NAL / slice layer
int Decoder::decode(const uint8_t* data, size_t size, h264p_output_fn out, void* user)
{
    out_ = out;
    user_ = user;
    stop_ = 0;
    err.clear();
    if (inflight_ >= 0) (void)h264r_picture_wait(ctx_, nullptr, nullptr, nullptr);  // left by a failed call
    inflight_ = -1;
    pending_.clear();
    pslices_.clear();
    try {
        // Annex-B: start codes 0x000001 (B.2); a NAL ends at the next start code (its
        // trailing_zero_8bits dropped)
        size_t i = 0;
        auto next_start = [&](size_t from) -> size_t {
            for (size_t k = from; k + 2 < size; ++k)
                if (data[k] == 0 && data[k + 1] == 0 && data[k + 2] == 1) return k;
            return size;
        };
        i = next_start(0);
        while (i < size && !stop_) {
            const size_t s = i + 3;
            size_t e = next_start(s);
            const size_t nxt = e;
            while (e > s && data[e - 1] == 0) --e;
            if (e > s) nal(data + s, e - s);
            i = nxt;
        }
        if (!stop_ && in_picture_) finish_picture();
        if (!stop_) flush_output();
    } catch (const Error& x) {
        err = x.what;
        return x.status;
    }
    return stop_;
}

void Decoder::nal(const uint8_t* p, size_t n)
{
    const int ref_idc = (p[0] >> 5) & 3, type = p[0] & 31;
    Bits b;
    switch (type) {
    case 1:
    case 5:
        b.load(p + 1, n - 1);
        slice(b, ref_idc, type);
        return;
    case 2: case 3: case 4:
        fail(H264R_EUNSUPPORTED, "data partitioning (NAL types 2-4)");
    case 7: {
        run_slices();                                  // the pending slices refer to the current sets
        b.load(p + 1, n - 1);
        Sps s;
        const int id = parse_sps(b, s);
        std::vector<uint8_t> raw(p + 1, p + n);
        if (sps_[id].valid && raw == sps_raw_[id]) return;          // a repeat of the stored set
        // a different set under the active id ends the open picture first, as the reference
        // calls exit_picture before activating it (slice_header.cc:392-423)
        if (in_picture_ && psps_ == &sps_[id]) finish_picture();
        sps_[id] = s;
        sps_raw_[id] = std::move(raw);
        return;
    }
    case 8: {
        run_slices();
        b.load(p + 1, n - 1);
        Pps q;
        const int id = parse_pps(b, q, sps_);
        std::vector<uint8_t> raw(p + 1, p + n);
        if (pps_[id].valid && raw == pps_raw_[id]) return;
        if (in_picture_ && pps_used_[id]) finish_picture();
        pps_[id] = q;
        pps_raw_[id] = std::move(raw);
        return;
    }
    case 11:                                      // end of stream
        if (in_picture_) finish_picture();
        return;
    default:                                      // SEI, AUD, end of sequence, filler, ...
        return;
    }
}

// slice_header (7.3.3; interpret_rbsp.cc:625-777)
void Decoder::parse_slice_header(Bits& b, SliceHeader& h)
{
    h.first_mb = b.ue_max(1024 * 1024 - 1, "slice: first_mb_in_slice");
    h.slice_type = b.ue_max(9, "slice: slice_type") % 5;
    h.pps_id = b.ue_max(255, "slice: pic_parameter_set_id");
    require(pps_[h.pps_id].valid, "slice: pic_parameter_set_id of no PPS");
    const Pps& pps = pps_[h.pps_id];
    const Sps& sps = sps_[pps.sps_id];
    unsupported(sps.separate_planes || sps.bit_depth_y != 8 || (sps.chroma_format_idc && sps.bit_depth_c != 8),
                "picture format (4:0:0, 4:2:0, 4:2:2 or 4:4:4 without separate colour planes, 8-bit only)");
    unsupported(sps.chroma_format_idc == 3 && pps.cabac, "4:4:4 with CABAC (entropy_coding_mode_flag)");
    // MBAFF with CABAC: the contexts are written (cabac_field_flag, the read-ahead of a skipped top MB's
    // bottom MB, refIdx / mvd across field and frame pairs) but the own parser does not yet reproduce the
    // reference on tests/streams.py's CABAC MBAFF streams, so they are refused (the shim path takes them)
    unsupported(sps.mbaff && pps.cabac, "MBAFF coding with CABAC");
    unsupported(sps.mbaff && h.slice_type == H264R_SLICE_B, "B slices of MBAFF frames");
    unsupported(sps.poc_type == 1, "pic_order_cnt_type 1");
    unsupported(h.slice_type == H264R_SLICE_SI, "SI slices");
    h.frame_num = b.u(sps.log2_max_frame_num);
    if (!sps.frame_mbs_only) {
        h.field = b.u(1);
        if (h.field) h.bottom = b.u(1);
        unsupported(h.field && sps.chroma_format_idc != 1, "4:2:2 / 4:4:4 field pictures");
    }
    if (h.idr) h.idr_pic_id = b.ue_max(65535, "slice: idr_pic_id");
    if (sps.poc_type == 0) {
        h.poc_lsb = b.u(sps.log2_max_poc_lsb);
        if (pps.bottom_field_poc && !h.field) h.delta_poc_bottom = b.se();
    }
    if (pps.redundant_pic_cnt) unsupported(b.ue_max(127, "slice: redundant_pic_cnt") != 0, "redundant pictures");
    const bool P = h.slice_type == H264R_SLICE_P || h.slice_type == H264R_SLICE_SP, B = h.slice_type == H264R_SLICE_B;
    if (B) h.direct_spatial = b.u(1);
    h.nref[0] = pps.nref_default[0];
    h.nref[1] = pps.nref_default[1];
    if (P || B) {
        if (b.u(1)) {
            h.nref[0] = b.ue_max(31, "slice: num_ref_idx_l0_active_minus1") + 1;
            if (B) h.nref[1] = b.ue_max(31, "slice: num_ref_idx_l1_active_minus1") + 1;
        }
        // frames: at most 16 per list (the reference asserts it, interpret_rbsp.cc:710;
        // H264R_MAX_REFS): a larger count would be clamped downstream, not decoded; fields: 32,
        // of which the reconstruction ABI takes 16
        require(h.nref[0] <= (h.field ? 32 : 16) && (!B || h.nref[1] <= (h.field ? 32 : 16)),
                "slice: num_ref_idx_active above 16 (frames) / 32 (fields)");
        unsupported(h.nref[0] > 16 || h.nref[1] > 16, "more than 16 reference fields in a list");
    }
    if (!B) h.nref[1] = 0;
    if (!P && !B) h.nref[0] = 0;
    // ref_pic_list_modification (7.3.3.1)
    for (int l = 0; l < (B ? 2 : P ? 1 : 0); ++l) {
        h.mod_flag[l] = b.u(1);
        unsupported(h.mod_flag[l] && h.field, "reference list modification in field pictures");
        if (h.mod_flag[l])
            for (;;) {
                const int idc = b.ue_max(3, "slice: modification_of_pic_nums_idc");
                if (idc == 3) break;
                // at most num_ref_idx_active entries (the reference asserts it,
                // interpret_rbsp.cc:803): each one writes a list entry
                require((int)h.mods[l].size() < h.nref[l], "slice: more list modifications than active references");
                h.mods[l].push_back({idc, b.ue_max(1u << 17, "slice: abs_diff_pic_num_minus1 / long_term_pic_num")});
            }
    }
    // pred_weight_table (7.3.3.2; interpret_rbsp.cc:832-905)
    if ((pps.weighted_pred && P) || (pps.weighted_bipred_idc == 1 && B)) {
        const bool chroma = sps.chroma_format_idc != 0;        // ChromaArrayType 0: luma weights only
        h.luma_log2_wd = b.ue_max(7, "slice: luma_log2_weight_denom");
        h.chroma_log2_wd = chroma ? b.ue_max(7, "slice: chroma_log2_weight_denom") : 0;   // absent: the header field stays 0
        for (int l = 0; l < (B ? 2 : 1); ++l)
            for (int i = 0; i < h.nref[l]; ++i) {
                h.weight[l][i][0] = 1 << h.luma_log2_wd;
                h.offset[l][i][0] = 0;
                if (b.u(1)) {
                    h.weight[l][i][0] = b.se_in(-128, 127, "slice: luma_weight");
                    h.offset[l][i][0] = b.se_in(-128, 127, "slice: luma_offset");
                }
                const bool cf = chroma && b.u(1);
                for (int j = 1; j < 3; ++j) {
                    h.weight[l][i][j] = chroma ? 1 << h.chroma_log2_wd : 0;      // 4:0:0: left 0, as the reference
                    h.offset[l][i][j] = 0;
                    if (cf) {
                        h.weight[l][i][j] = b.se_in(-128, 127, "slice: chroma_weight");
                        h.offset[l][i][j] = b.se_in(-128, 127, "slice: chroma_offset");
                    }
                }
            }
    }
    // dec_ref_pic_marking (7.3.3.3)
    if (h.nal_ref_idc) {
        if (h.idr) {
            h.no_output_of_prior_pics = b.u(1);
            h.long_term_reference = b.u(1);
        } else {
            h.adaptive = b.u(1);
            unsupported(h.adaptive && h.field, "adaptive reference marking in field pictures");
            if (h.adaptive)
                for (;;) {
                    Mmco m{b.ue_max(6, "slice: memory_management_control_operation"), 0, 0};
                    if (m.op == 0) break;
                    unsupported(m.op == 5, "MMCO 5");
                    require(h.mmco.size() < 64, "slice: memory_management_control_operation count");
                    if (m.op == 1 || m.op == 3) m.a = b.ue_max(1u << 17, "slice: difference_of_pic_nums_minus1");
                    if (m.op == 2) m.a = b.ue_max(1u << 17, "slice: long_term_pic_num");
                    if (m.op == 3 || m.op == 6) m.b = b.ue_max(15, "slice: long_term_frame_idx");
                    if (m.op == 4) m.a = b.ue_max(16, "slice: max_long_term_frame_idx_plus1");
                    h.mmco.push_back(m);
                }
        }
    }
    if (pps.cabac && h.slice_type != H264R_SLICE_I) {
        h.cabac_init_idc = b.ue_max(2, "slice: cabac_init_idc");
    }
    h.qp = pps.init_qp + b.se_in(-51, 51, "slice: slice_qp_delta");
    if (h.slice_type == H264R_SLICE_SP) {
        h.sp_switch = b.u(1);
        h.qs = pps.init_qs + b.se_in(-51, 51, "slice: slice_qs_delta");
    }
    require(h.qp >= 0 && h.qp <= 51 && h.qs >= 0 && h.qs <= 51, "slice: QP out of range");
    if (pps.deblocking_control) {
        h.deblock_idc = b.ue_max(2, "slice: disable_deblocking_filter_idc");
        if (h.deblock_idc != 1) {
            // the reference asserts -6..6 (interpret_rbsp.cc:760-765)
            h.offset_a = b.se_in(-6, 6, "slice: slice_alpha_c0_offset_div2") * 2;
            h.offset_b = b.se_in(-6, 6, "slice: slice_beta_offset_div2") * 2;
        }
    }
}

void Decoder::slice(Bits& b, int nal_ref_idc, int nal_type)
{
    SliceHeader h;
    h.nal_ref_idc = nal_ref_idc;
    h.nal_type = nal_type;
    h.idr = nal_type == 5;
    parse_slice_header(b, h);
    // first VCL NAL unit of a new picture (7.4.1.2.4)
    const bool new_pic = !in_picture_ || h.first_mb == 0 || h.frame_num != first_.frame_num ||
                         h.pps_id != first_.pps_id || (h.nal_ref_idc == 0) != (first_.nal_ref_idc == 0) ||
                         h.idr != first_.idr || (h.idr && h.idr_pic_id != first_.idr_pic_id) ||
                         h.poc_lsb != first_.poc_lsb || h.delta_poc_bottom != first_.delta_poc_bottom ||
                         h.field != first_.field || h.bottom != first_.bottom;
    if (new_pic) {
        if (in_picture_) finish_picture();
        if (stop_) return;
        begin_picture(h);
    }
    const Pps& pps = pps_[h.pps_id];
    const Sps& sps = sps_[pps.sps_id];
    require(&sps == psps_, "slice: SPS changes inside a picture");
    pps_used_[h.pps_id] = true;
    unsupported((int)slice_tab_.size() >= H264R_MAX_SLICES, "slices per picture");
    init_lists(h);
    slice_tab_.push_back(slice_record(h));
    const h264r_quant q = quant_tables(sps, pps);
    if (have_quant_ && memcmp(&quant_, &q, sizeof(q)) != 0)
        fail(H264R_EUNSUPPORTED, "scaling matrices differing between slices of one picture");
    quant_ = q;
    have_quant_ = true;
    auto ps = std::make_unique<PendingSlice>();
    ps->h = h;
    ps->b = std::move(b);
    ps->nr = (int)slice_tab_.size() - 1;
    ps->sps = &sps;
    ps->pps = &pps;
    memcpy(ps->list, list_, sizeof(list_));
    memcpy(ps->list_n, list_n_, sizeof(list_n_));
    pslices_.push_back(std::move(ps));
}

void Decoder::run_slices()
{
    const size_t n = pslices_.size();
    if (!n) return;
    const int W = psps_->W, H = pic_h_;
    static const int env_threads = [] {
        const char* e = getenv("H264P_THREADS");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    const int hw = std::max(1, (int)std::thread::hardware_concurrency());
    // threads pay off on large pictures; H264P_THREADS forces them (the tests use it)
    int threads = env_threads ? env_threads : (W * H >= 1200 ? std::min(8, hw) : 1);
    if (psps_->mbaff) threads = 1;                          // MBAFF slices: in order (their lookups reach later pairs)
    threads = std::min<int>(threads, (int)n);
    bool ordered = true;
    for (size_t k = 1; k < n; ++k) ordered &= pslices_[k - 1]->h.first_mb < pslices_[k]->h.first_mb;
    auto end_of = [&](size_t k) { return k + 1 < n ? pslices_[k + 1]->h.first_mb : W * H; };
    auto run_one = [&](size_t k, int end) {
        PendingSlice& p = *pslices_[k];
        SliceCtx sc(*this, *p.sps, *p.pps, p.h, p.nr, p.b, p.list, p.list_n, end);
        sc.run();
    };
    if (threads <= 1 || !ordered) {
        for (size_t k = 0; k < n; ++k) run_one(k, W * H);
        pslices_.clear();
        return;
    }
    // every MB's slice before the slices run, so an availability check never reads a slice
    // number another thread is writing (the neighbours of an MB precede it in raster order)
    for (size_t k = 0; k < n; ++k)
        for (int a = std::min(pslices_[k]->h.first_mb, W * H); a < std::min(end_of(k), W * H); ++a) mbs_[a].slice_nr = pslices_[k]->nr;
    std::atomic<size_t> next{0};
    std::vector<Error> errs(n);
    std::vector<uint8_t> failed(n, 0);
    auto worker = [&]() {
        for (;;) {
            const size_t k = next++;
            if (k >= n) return;
            try {
                run_one(k, end_of(k));
            } catch (const Error& e) {
                errs[k] = e;
                failed[k] = 1;
            } catch (const std::bad_alloc&) {
                errs[k] = Error{H264R_ENOMEM, "out of memory"};
                failed[k] = 1;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(worker);
    worker();
    for (auto& t : pool) t.join();
    pslices_.clear();
    for (size_t k = 0; k < n; ++k)
        if (failed[k]) throw errs[k];                 // the first slice's error, as the sequential order
}

// POC (8.2.1.1 type 0, 8.2.1.3 type 2) and the per-picture state (slice_data.cc init_picture)
void Decoder::begin_picture(const SliceHeader& h)
{
    const Pps& pps = pps_[h.pps_id];
    const Sps& sps = sps_[pps.sps_id];
    const int W = sps.W, H = sps.H;
    // the picture still on the GPU leaves the context (at its own size, Output::W/H) before the
    // context is replaced for a larger picture size
    if (!ctx_ || W > ctx_w_ || H > ctx_h_ || sps.chroma_format_idc != ctx_cf_) collect();
    psps_ = &sps;
    ppps_ = &pps;
    first_ = h;
    in_picture_ = true;
    pps_used_.reset();
    if (!ctx_ || W > ctx_w_ || H > ctx_h_ || sps.chroma_format_idc != ctx_cf_) {
        if (ctx_) h264r_destroy(ctx_);
        ctx_ = nullptr;
        for (auto& p : dpb_) p->slot = -1;
        check(h264r_create(&ctx_, device_, W, H, sps.chroma_format_idc, 8), "h264r_create");
        ctx_w_ = W;
        ctx_h_ = H;
        ctx_cf_ = sps.chroma_format_idc;
    }
    if (W != mbs_w_ || H != mbs_h_) {            // the reference's mb_data (init_global_buffers)
        mbs_.assign((size_t)W * H, MbState());
        mbs_w_ = W;
        mbs_h_ = H;
    }
    // MBAFF: a neighbour lookup may land in a later pair of this picture (the bottom MB of the
    // current pair, the pair to the right), which must read as not decoded (reset_mbs,
    // slice_data.cc:53-58)
    if (sps.mbaff)
        for (MbState& m : mbs_) { m.slice_nr = -1; m.fld = false; }
    unsupported(sps.gaps, "gaps_in_frame_num_value_allowed_flag");
    int poc = 0;
    const int max_frame_num = 1 << sps.log2_max_frame_num;
    if (sps.poc_type == 0) {
        if (h.idr) { prev_poc_msb_ = 0; prev_poc_lsb_ = 0; }
        const int max_lsb = 1 << sps.log2_max_poc_lsb;
        int msb;
        if (h.poc_lsb < prev_poc_lsb_ && prev_poc_lsb_ - h.poc_lsb >= max_lsb / 2) msb = prev_poc_msb_ + max_lsb;
        else if (h.poc_lsb > prev_poc_lsb_ && h.poc_lsb - prev_poc_lsb_ > max_lsb / 2) msb = prev_poc_msb_ - max_lsb;
        else msb = prev_poc_msb_;
        // a field picture: its own lsb gives its field's count (8.2.1.1); a frame: both
        const int top = msb + h.poc_lsb, bottom = h.field ? top : top + h.delta_poc_bottom;
        poc = std::min(top, bottom);
        if (h.nal_ref_idc) { prev_poc_msb_ = msb; prev_poc_lsb_ = h.poc_lsb; }
    } else {
        int offset;
        if (h.idr) offset = 0;
        else if (prev_frame_num_ > h.frame_num) offset = prev_frame_num_offset_ + max_frame_num;
        else offset = prev_frame_num_offset_;
        poc = h.idr ? 0 : h.nal_ref_idc ? 2 * (offset + h.frame_num) : 2 * (offset + h.frame_num) - 1;
        prev_frame_num_offset_ = offset;
    }
    prev_frame_num_ = h.frame_num;
    cur_poc_ = poc;
    pic_h_ = h.field ? H / 2 : H;
    const int par = h.bottom ? 1 : 0;
    // the second field of a frame store: the stored field of the opposite parity, the same
    // frame_num, both reference fields or both not (the pairing of store_picture dpb.cc:903-912)
    if (last_field_) {
        const bool pair = h.field && !h.idr && last_field_->frame_num == h.frame_num && !last_field_->has[par] &&
                          last_field_->ref == (h.nal_ref_idc != 0);
        unsupported(!pair, "an unpaired field");
        cur_ = last_field_;
        cur_->poc_f[par] = poc;
        cur_->poc = std::min(cur_->poc_f[0], cur_->poc_f[1]);
    } else {
        if (h.idr) {
            flush_output();
            ++period_;
        }
        auto pic = std::make_unique<Picture>();
        pic->id = next_id_++;
        pic->poc = poc;
        pic->frame_num = h.frame_num;
        pic->idr = h.idr;
        pic->ref = h.nal_ref_idc != 0;
        pic->fields = h.field;
        pic->poc_f[0] = pic->poc_f[1] = poc;
        if (h.field) {
            pic->has[0] = par == 0;
            pic->has[1] = par == 1;
        }
        cur_ = pic.get();
        dpb_.push_back(std::move(pic));
    }
    mot_ = std::make_shared<Motion>();
    mot_->init(W, pic_h_);
    if (!h.field) cur_->mot = mot_;
    else cur_->mot_f[par] = mot_;
    staged_.assign((size_t)W * pic_h_, StagedMb());
    seen_.assign((size_t)W * pic_h_, 0);
    slice_tab_.clear();
    have_quant_ = false;
}

// RefPicList0/1 (slice_ref_list.cc:88-341) and their modification (:885-964), frames only
void Decoder::init_lists(const SliceHeader& h)
{
    const int max_frame_num = 1 << psps_->log2_max_frame_num;
    std::vector<Picture*> st, lt;
    if (h.field) {
        init_field_lists(h);
        return;
    }
    for (auto& p : dpb_) {
        if (p.get() == cur_ || !p->ref) continue;
        // a frame's list holds frame stores whose two fields are both reference fields
        // (init_lists_p_slice slice_ref_list.cc:93-99: is_used == 3, frame used for reference)
        if (!p->has[0] || !p->has[1] || !p->ref_f[0] || !p->ref_f[1]) continue;
        if (p->long_term) lt.push_back(p.get());
        else {
            p->frame_num_wrap = p->frame_num > h.frame_num ? p->frame_num - max_frame_num : p->frame_num;
            st.push_back(p.get());
        }
    }
    std::sort(lt.begin(), lt.end(), [](Picture* a, Picture* b) { return a->lt_idx < b->lt_idx; });
    list_n_[0] = list_n_[1] = 0;
    for (int l = 0; l < 2; ++l)
        for (int i = 0; i < 33; ++i) list_[l][i] = nullptr;
    if (h.slice_type == H264R_SLICE_P || h.slice_type == H264R_SLICE_SP) {
        std::sort(st.begin(), st.end(), [](Picture* a, Picture* b) { return a->frame_num_wrap > b->frame_num_wrap; });
        int n = 0;
        for (Picture* p : st) list_[0][n++] = p;
        for (Picture* p : lt) list_[0][n++] = p;
        list_n_[0] = n;
    } else if (h.slice_type == H264R_SLICE_B) {
        const int poc = cur_->poc;
        std::vector<Picture*> before, after;
        for (Picture* p : st) (poc >= p->poc ? before : after).push_back(p);
        std::sort(before.begin(), before.end(), [](Picture* a, Picture* b) { return a->poc > b->poc; });
        std::sort(after.begin(), after.end(), [](Picture* a, Picture* b) { return a->poc < b->poc; });
        int n = 0;
        for (Picture* p : before) list_[0][n++] = p;
        for (Picture* p : after) list_[0][n++] = p;
        int m = 0;
        for (Picture* p : after) list_[1][m++] = p;
        for (Picture* p : before) list_[1][m++] = p;
        for (Picture* p : lt) { list_[0][n++] = p; list_[1][m++] = p; }
        list_n_[0] = n;
        list_n_[1] = m;
        if (n == m && n > 1) {
            bool same = true;
            for (int j = 0; j < n; ++j) same &= list_[0][j] == list_[1][j];
            if (same) std::swap(list_[1][0], list_[1][1]);
        }
    }
    for (int l = 0; l < 2; ++l) {
        list_n_[l] = std::min(list_n_[l], h.nref[l]);
        for (int i = list_n_[l]; i < 33; ++i) list_[l][i] = nullptr;
        if (h.mod_flag[l]) modify_list(h, l);
        // RefPicSize = num_ref_idx_active (:949, :962): every entry must name a picture
        // (the shim refuses a non-resident one)
        list_n_[l] = h.nref[l];
        for (int i = 0; i < list_n_[l]; ++i)
            require(list_[l][i] != nullptr, "RefPicList entry is 'no reference picture'");
    }
}

// RefPicList0 of a P field (8.2.4.2.5; init_lists_p_slice slice_ref_list.cc:128-170,
// gen_pic_list_from_frame_list :18-76): the frame stores with a short-term reference field --
// the current frame's first field included -- by FrameNumWrap, descending, then the long-term
// ones by LongTermFrameIdx; from each ordered set the fields alternate, same parity first, and
// a parity that runs out leaves the rest to the other
void Decoder::init_field_lists(const SliceHeader& h)
{
    const int max_frame_num = 1 << psps_->log2_max_frame_num;
    std::vector<Picture*> st, lt;
    for (auto& p : dpb_) {
        const bool r = (p->has[0] && p->ref_f[0]) || (p->has[1] && p->ref_f[1]);
        if (!p->ref || !r) continue;
        if (p.get() == cur_ && !p->fields) continue;
        if (p->long_term) lt.push_back(p.get());
        else {
            p->frame_num_wrap = p->frame_num > h.frame_num ? p->frame_num - max_frame_num : p->frame_num;
            st.push_back(p.get());
        }
    }
    std::sort(lt.begin(), lt.end(), [](Picture* a, Picture* b) { return a->lt_idx < b->lt_idx; });
    list_n_[0] = list_n_[1] = 0;
    for (int l = 0; l < 2; ++l)
        for (int i = 0; i < 33; ++i) list_[l][i] = nullptr;
    const int same = h.bottom ? 1 : 0;
    // the fields of the ordered frame stores fs appended to list l, alternating parity
    auto gen = [&](const std::vector<Picture*>& fs, int l) {
        size_t idx[2] = {0, 0};
        auto next = [&](int k) {                    // the next frame store holding a reference field k
            for (; idx[k] < fs.size(); ++idx[k])
                if (fs[idx[k]]->has[k] && fs[idx[k]]->ref_f[k]) {
                    if (list_n_[l] < 32) list_[l][list_n_[l]++] = fs[idx[k]]->field(k, next_id_);
                    ++idx[k];
                    return;
                }
        };
        while (idx[0] < fs.size() || idx[1] < fs.size()) {
            next(same);
            next(1 - same);
        }
    };
    if (h.slice_type != H264R_SLICE_B) {
        std::sort(st.begin(), st.end(), [](Picture* a, Picture* b) { return a->frame_num_wrap > b->frame_num_wrap; });
        gen(st, 0);
        gen(lt, 0);
    } else {
        // B fields (init_lists_b_slice slice_ref_list.cc:256-306): the frame stores by their POC
        // (a single field's, or the pair's smaller) against the current field's -- list 0 those
        // at or before it (descending) then after (ascending), list 1 the two halves swapped
        std::vector<Picture*> before, after, l0, l1;
        for (Picture* p : st) (cur_poc_ >= p->poc ? before : after).push_back(p);
        std::stable_sort(before.begin(), before.end(), [](Picture* a, Picture* b) { return a->poc > b->poc; });
        std::stable_sort(after.begin(), after.end(), [](Picture* a, Picture* b) { return a->poc < b->poc; });
        l0 = before; l0.insert(l0.end(), after.begin(), after.end());
        l1 = after; l1.insert(l1.end(), before.begin(), before.end());
        gen(l0, 0);
        gen(l1, 1);
        gen(lt, 0);
        gen(lt, 1);
        if (list_n_[0] == list_n_[1] && list_n_[0] > 1) {
            bool identical = true;
            for (int j = 0; j < list_n_[0]; ++j) identical &= list_[0][j] == list_[1][j];
            if (identical) std::swap(list_[1][0], list_[1][1]);
        }
    }
    for (int l = 0; l < 2; ++l) {
        list_n_[l] = std::min(list_n_[l], h.nref[l]);
        for (int i = list_n_[l]; i < 33; ++i) list_[l][i] = nullptr;
        list_n_[l] = h.nref[l];
        for (int i = 0; i < list_n_[l]; ++i) require(list_[l][i] != nullptr, "RefPicList entry is 'no reference picture'");
    }
}

void Decoder::modify_list(const SliceHeader& h, int l)
{
    const int max_pic_num = 1 << psps_->log2_max_frame_num, curr = h.frame_num;
    const int n = h.nref[l];
    Picture** L = list_[l];
    int pred = curr, ref_idx = 0;
    for (const ListMod& m : h.mods[l]) {
        Picture* pic = nullptr;
        int pic_num = 0;
        if (m.idc < 2) {
            const int d = m.val + 1;
            int no_wrap;
            if (m.idc == 0) no_wrap = pred - d < 0 ? pred - d + max_pic_num : pred - d;
            else no_wrap = pred + d >= max_pic_num ? pred + d - max_pic_num : pred + d;
            pred = no_wrap;
            pic_num = no_wrap > curr ? no_wrap - max_pic_num : no_wrap;
            for (auto& p : dpb_)
                if (p.get() != cur_ && p->ref && !p->long_term && p->frame_num_wrap == pic_num) pic = p.get();
        } else {
            for (auto& p : dpb_)
                if (p.get() != cur_ && p->ref && p->long_term && p->lt_idx == m.val) pic = p.get();
        }
        require(pic != nullptr, "ref_pic_list_modification names no reference picture");
        for (int c = n; c > ref_idx; --c) L[c] = L[c - 1];
        L[ref_idx++] = pic;
        int k = ref_idx;
        for (int c = ref_idx; c <= n; ++c)
            if (L[c] && L[c] != pic) L[k++] = L[c];
        for (; k <= n; ++k) L[k] = nullptr;
    }
}

// h264r_slice of the slice (the shim's slice_record, decoder_h264r.cc:160-224)
h264r_slice Decoder::slice_record(const SliceHeader& h)
{
    h264r_slice r;
    memset(&r, 0, sizeof(r));
    const Pps& pps = *ppps_;
    r.slice_type = (uint8_t)h.slice_type;
    r.qs_y = (uint8_t)h.qs;
    r.sp_switch = h.sp_switch ? 1 : 0;
    r.deblock_idc = (uint8_t)h.deblock_idc;
    r.filter_offset_a = (int8_t)h.offset_a;
    r.filter_offset_b = (int8_t)h.offset_b;
    const bool P = h.slice_type == H264R_SLICE_P || h.slice_type == H264R_SLICE_SP, B = h.slice_type == H264R_SLICE_B;
    r.wp_mode = (pps.weighted_pred && P) || (pps.weighted_bipred_idc == 1 && B) ? 1 : (pps.weighted_bipred_idc == 2 && B) ? 2 : 0;
    r.luma_log2_wd = (uint8_t)(r.wp_mode == 1 ? h.luma_log2_wd : 5);
    r.chroma_log2_wd = (uint8_t)(r.wp_mode == 1 ? h.chroma_log2_wd : 5);
    for (int l = 0; l < 2; ++l) {
        const int n = std::min(list_n_[l], H264R_MAX_REFS);
        r.num_ref[l] = (uint8_t)n;
        for (int i = 0; i < H264R_MAX_REFS; ++i) {
            r.ref_slot[l][i] = -1;
            if (i < n && list_[l][i]) {
                // a field view names its frame store's slot and its parity (include/h264r.h)
                const Picture* q = list_[l][i]->parent ? list_[l][i]->parent : list_[l][i];
                if (q->slot < 0) fail(H264R_ESTATE, "reference picture not resident in a device DPB slot");
                r.ref_slot[l][i] = (int8_t)(q->slot | (list_[l][i]->parent && list_[l][i]->parity ? H264R_REF_BOTTOM : 0));
            }
            if (r.wp_mode == 1 && i < h.nref[l])
                for (int pl = 0; pl < 3; ++pl) {
                    r.wp_weight[l][i][pl] = (int8_t)h.weight[l][i][pl];
                    r.wp_offset[l][i][pl] = (int8_t)h.offset[l][i][pl];
                }
        }
    }
    if (r.wp_mode == 2)                                   // implicit weights (inter_prediction.cc:112-139)
        for (int i0 = 0; i0 < r.num_ref[0]; ++i0)
            for (int i1 = 0; i1 < r.num_ref[1]; ++i1) {
                const Picture* p0 = list_[0][i0];
                const Picture* p1 = list_[1][i1];
                int w1 = 32;
                if (p0 && p1) {
                    const int td = clip3(-128, 127, p1->poc - p0->poc);
                    if (td != 0 && !p0->long_term && !p1->long_term) {
                        const int tb = clip3(-128, 127, cur_poc_ - p0->poc);
                        const int tx = (16384 + std::abs(td / 2)) / td;
                        const int dsf = clip3(-1024, 1023, (tx * tb + 32) >> 6);
                        w1 = dsf >> 2;
                        if (w1 < -64 || w1 > 128) w1 = 32;
                    }
                }
                r.implicit_w1[i0][i1] = (int16_t)w1;
            }
    return r;
}

// Reconstruction of the picture through the h264r ABI (the shim's deblock_filter,
// decoder_h264r.cc:470-533), then marking (8.2.5) and output.
void Decoder::finish_picture()
{
    run_slices();
    in_picture_ = false;
    const int W = psps_->W, H = pic_h_;
    const bool fld = first_.field, second = fld && cur_ == last_field_;
    const int par = first_.bottom ? 1 : 0;
    if (!have_quant_) check(h264r_quant_init_flat(&quant_), "h264r_quant_init_flat");
    h264r_pic p;
    memset(&p, 0, sizeof(p));
    p.constrained_intra_pred = ppps_->cip;
    p.num_slices = (int)slice_tab_.size();
    p.poc = cur_poc_;
    p.structure = !fld ? (psps_->mbaff ? H264R_MBAFF_FRAME : H264R_FRAME) : par ? H264R_BOTTOM_FIELD : H264R_TOP_FIELD;
    check(h264r_picture_begin(ctx_, W, H, &p, slice_tab_.data(), &quant_), "h264r_picture_begin");
    for (int a = 0; a < W * H; ++a) {
        if (!seen_[a]) fail(H264R_ESTATE, "picture with missing macroblocks");
        StagedMb& st = staged_[a];
        check(h264r_mb_submit(ctx_, a, &st.rec, st.levels.empty() ? nullptr : st.levels.data(), (int)st.levels.size(),
                              &st.mv[0][0], &st.ref[0][0]), "h264r_mb_submit");
    }
    int keep = -1;
    if (second) keep = cur_->slot;                     // the second field: its first field's slot
    else if (cur_->ref) {
        // a device slot no reference picture holds, round robin (the shim's policy: the
        // references as they stand before this picture's own marking)
        bool busy[H264R_MAX_SLOTS] = {};
        for (auto& q : dpb_)
            if (q.get() != cur_ && q->ref && q->slot >= 0) busy[q->slot] = true;
        for (int k = 0; k < H264R_MAX_SLOTS && keep < 0; ++k)
            if (!busy[(next_slot_ + k) % H264R_MAX_SLOTS]) keep = (next_slot_ + k) % H264R_MAX_SLOTS;
        if (keep < 0) fail(H264R_EUNSUPPORTED, "more than 32 reference frames resident");
        next_slot_ = (keep + 1) % H264R_MAX_SLOTS;
        for (auto& q : dpb_)
            if (q->slot == keep) q->slot = -1;
    }
    // the output frame: a field pair's second field fills the other rows of its first field's
    // entry (dpb_combine_field_yuv picture.cc:578-622), whose POC is the pair's smaller one
    const int FH = fld ? 2 * H : H;
    // (vertical crop offsets count 2 chroma rows when the stream may hold fields, CropUnitY)
    const int cuy = psps_->frame_mbs_only ? 1 : 2;
    if (!second)
        pending_.push_back(Output{period_, cur_->poc, W, FH,
                                  {psps_->crop[0], psps_->crop[1], cuy * psps_->crop[2], cuy * psps_->crop[3]}, {}, {}, {},
                                  psps_->chroma_format_idc});
    const int out_idx = second ? out_of_first_ : (int)pending_.size() - 1;
    pending_[out_idx].poc = cur_->poc;
    if (sync_) {
        collect();
        check(h264r_picture_end_async(ctx_, keep), "h264r_picture_end_async");
        inflight_ = out_idx;
        inflight_par_ = fld ? par : -1;
        collect();
    } else {
        // this picture is reconstructed while the next one is parsed; the previous one is
        // collected now (the h264r ABI stages two pictures)
        check(h264r_picture_end_async(ctx_, keep), "h264r_picture_end_async");
        collect();
        inflight_ = out_idx;
        inflight_par_ = fld ? par : -1;
    }
    cur_->slot = keep;
    mark_picture();
    last_field_ = fld && !second ? cur_ : nullptr;
    if (fld && !second) out_of_first_ = out_idx;
    // pictures no longer used for reference leave the DPB (their motion with them)
    // (a non-reference first field stays for its second field)
    dpb_.erase(std::remove_if(dpb_.begin(), dpb_.end(),
                              [&](const std::unique_ptr<Picture>& q) { return !q->ref && q.get() != last_field_; }),
               dpb_.end());
    cur_ = nullptr;
}

// Decoded reference picture marking (8.2.5; dpb.cc idr_memory_management,
// sliding_window_memory_management, adaptive_memory_management)
void Decoder::mark_picture()
{
    if (!cur_->ref) return;
    const SliceHeader& h = first_;
    struct Norm {                                  // per-field marking follows the frame store's
        Decoder& d;
        ~Norm()
        {
            for (auto& q : d.dpb_) {
                if (!q->fields) q->ref_f[0] = q->ref_f[1] = q->ref;
                else if (!q->ref) q->ref_f[0] = q->ref_f[1] = false;
            }
        }
    } norm{*this};
    if (h.field) {
        cur_->ref_f[h.bottom ? 1 : 0] = true;
        cur_->has[h.bottom ? 1 : 0] = true;
        // the second field of a pair: no sliding window (store_picture dpb.cc:903-912 stores it
        // into its first field's frame store before the window runs)
        if (cur_ == last_field_) return;
    }
    auto others = [&](auto fn) {
        for (auto& q : dpb_)
            if (q.get() != cur_ && q->ref) fn(*q);
    };
    if (h.idr) {
        others([](Picture& q) { q.ref = false; });
        if (h.long_term_reference) {
            cur_->long_term = true;
            cur_->lt_idx = 0;
            max_lt_idx_ = 0;
        } else
            max_lt_idx_ = -1;
        return;
    }
    const int max_frame_num = 1 << psps_->log2_max_frame_num, curr = h.frame_num;
    others([&](Picture& q) {
        if (!q.long_term) q.frame_num_wrap = q.frame_num > curr ? q.frame_num - max_frame_num : q.frame_num;
    });
    bool cur_lt = false;
    if (h.adaptive) {
        for (const Mmco& m : h.mmco) {
            switch (m.op) {
            case 1: {
                const int num = curr - (m.a + 1);
                others([&](Picture& q) { if (!q.long_term && q.frame_num_wrap == num) q.ref = false; });
                break;
            }
            case 2:
                others([&](Picture& q) { if (q.long_term && q.lt_idx == m.a) q.ref = false; });
                break;
            case 3: {
                const int num = curr - (m.a + 1);
                others([&](Picture& q) { if (q.long_term && q.lt_idx == m.b) q.ref = false; });
                others([&](Picture& q) {
                    if (!q.long_term && q.frame_num_wrap == num) { q.long_term = true; q.lt_idx = m.b; }
                });
                break;
            }
            case 4:
                max_lt_idx_ = m.a - 1;
                others([&](Picture& q) { if (q.long_term && q.lt_idx > max_lt_idx_) q.ref = false; });
                break;
            case 6:
                others([&](Picture& q) { if (q.long_term && q.lt_idx == m.b) q.ref = false; });
                cur_lt = true;
                cur_->long_term = true;
                cur_->lt_idx = m.b;
                break;
            }
        }
    } else {
        int n = 0;
        Picture* oldest = nullptr;
        others([&](Picture& q) {
            ++n;
            if (!q.long_term && (!oldest || q.frame_num_wrap < oldest->frame_num_wrap)) oldest = &q;
        });
        if (n >= std::max(1, psps_->max_num_ref_frames) && oldest) oldest->ref = false;
    }
    (void)cur_lt;
}

// Planes of the picture still on the GPU into its output entry.
void Decoder::collect()
{
    if (inflight_ < 0) return;
    Output& o = pending_[inflight_];
    inflight_ = -1;
    const size_t n = (size_t)o.W * o.H, cs = n * (o.cf == 3 ? 256 : o.cf == 2 ? 128 : o.cf == 1 ? 64 : 0);
    if (o.y.size() != n * 256 || o.u.size() != cs) {
        o.y.assign(n * 256, 0);
        o.u.assign(cs, 0);
        o.v.assign(cs, 0);
    }
    if (inflight_par_ < 0) {
        check(h264r_picture_wait(ctx_, o.y.data(), o.u.data(), o.v.data()), "h264r_picture_wait");
        return;
    }
    // a field: its rows of the frame (every second row from row `par`)
    const int par = inflight_par_;
    inflight_par_ = -1;
    fy_.resize(n * 128);
    fu_.resize(n * 32);
    fv_.resize(n * 32);
    check(h264r_picture_wait(ctx_, fy_.data(), fu_.data(), fv_.data()), "h264r_picture_wait");
    const int w = o.W * 16, wc = o.W * 8;
    for (int r = 0; r < o.H * 8; ++r) memcpy(&o.y[(size_t)(2 * r + par) * w], &fy_[(size_t)r * w], w);
    for (int r = 0; r < o.H * 4; ++r) {
        memcpy(&o.u[(size_t)(2 * r + par) * wc], &fu_[(size_t)r * wc], wc);
        memcpy(&o.v[(size_t)(2 * r + par) * wc], &fv_[(size_t)r * wc], wc);
    }
}

void Decoder::flush_output()
{
    collect();
    std::stable_sort(pending_.begin(), pending_.end(),
                     [](const Output& a, const Output& b) { return a.period != b.period ? a.period < b.period : a.poc < b.poc; });
    for (Output& o : pending_) {
        if (stop_) break;
        h264p_frame f;
        f.y = o.y.data(); f.u = o.u.data(); f.v = o.v.data();
        f.width = o.W * 16;
        f.height = o.H * 16;
        const int sub_h = o.cf == 1 ? 2 : 1, sub_w = o.cf == 1 || o.cf == 2 ? 2 : 1;   // CropUnitY / X per crop unit
        f.crop_left = sub_w * o.crop[0]; f.crop_right = sub_w * o.crop[1];
        f.crop_top = sub_h * o.crop[2]; f.crop_bottom = sub_h * o.crop[3];
        f.chroma_format = o.cf;
        f.poc = o.poc;
        f.period = o.period;
        if (out_) stop_ = out_(user_, &f);
    }
    pending_.clear();
}

// ------------------------------------------------------------------ macroblock layer
SliceCtx::SliceCtx(Decoder& d, const Sps& s, const Pps& p, const SliceHeader& h, int nr, Bits& bits,
                   Picture* const (*lists)[33], const int* list_n, int end)
    : D(d), sps(s), pps(p), sh(h), slice_nr(nr), b(bits), W(s.W), H(h.field ? s.H / 2 : s.H),
      cf(s.chroma_format_idc), mwc(s.chroma_format_idc == 3 ? 16 : s.chroma_format_idc ? 8 : 0),
      mhc(s.chroma_format_idc == 1 ? 8 : s.chroma_format_idc ? 16 : 0),
      zz4(h.field ? FIELD_SCAN4X4 : ZZ4), zz8(h.field ? FIELD_SCAN8X8 : ZZ8), qp(h.qp),
      mbaff(s.mbaff && !h.field), list_(lists), list_n_(list_n), end_mb(end)
{
}

// slice_data (7.3.4; slice_data.cc:636-660, macroblock_t::close :526-565)
void SliceCtx::run()
{
    const bool I = sh.slice_type == H264R_SLICE_I;
    addr = sh.first_mb * (mbaff ? 2 : 1);                   // MBAFF: first_mb_in_slice counts MB pairs
    require(addr < W * H, "slice: first_mb_in_slice");
    if (pps.cabac) {
        // Parser::init / slice_t::init (interpret_mb.cc:138-156, slice_data.cc:602-604); the
        // end_of_slice_flag after every MB but the picture's last (macroblock_t::close :526-565)
        static thread_local Cabac engine;
        cab = &engine;
        const int kind = I ? 0 : (sh.slice_type == H264R_SLICE_B ? 4 : 1) + sh.cabac_init_idc;
        cab->init_contexts(kind, sh.qp);
        cab->init_engine(b);
        for (;;) {
            macroblock();
            if (addr == W * H - 1) { cab->check_end(); return; }
            if (mbaff && !(addr & 1)) { ++addr; continue; }      // MBAFF: end_of_slice_flag after bottom MBs only (:531)
            const int eos = cab->term();
            ++addr;
            if (eos) return;
            require(addr < end_mb, "slice: runs into the next slice");
        }
    }
    for (;;) {
        macroblock();
        if (addr == W * H - 1) return;
        ++addr;
        if (!b.more_rbsp_data() && (I || skip_run <= 0)) return;
        require(addr < end_mb, "slice: runs into the next slice");
    }
}

void SliceCtx::update_qp(int q)
{
    qpy = q;
    qp_scaled[0] = q;
    for (int i = 0; i < 2; ++i) {
        const int qpi = clip3(0, 51, q + pps.cqp_offset[i]);
        qpc[i] = qpi < 30 ? qpi : QP_SCALE_CR[qpi];
        qp_scaled[i + 1] = qpc[i];
        const int qsi = clip3(0, 51, sh.qs + pps.cqp_offset[i]);
        qsc[i] = qsi < 30 ? qsi : QP_SCALE_CR[qsi];
    }
    bypass = sps.bypass && qp_scaled[0] == 0;
}

// the MB covering (xN, yN) relative to the current MB's top-left sample (luma or chroma
// units), if inside the picture and of the current slice (neighbour.cc:123-173 + the
// callers' slice_nr checks); ax, ay = absolute sample position
MbState* SliceCtx::nb_mb(bool chroma, int xN, int yN, int& ax, int& ay)
{
    const int mw = chroma ? mwc : 16, mh = chroma ? mhc : 16;
    if (mbaff) {
        // MBAFF (neighbour.cc:123-173): the geometric frame sample of the current MB's (xN, yN) -- a
        // field MB's rows are every second row of its pair --, the MB holding it (the bottom MB of a
        // field pair for odd rows, of a frame pair for its lower half) and the sample's storage
        // position in that MB's rows (ax, ay)
        const int lx = mbx * mw + xN;
        const int ly = (mby >> 1) * 2 * mh + (cur->fld ? (mby & 1) + 2 * yN : (mby & 1) * mh + yN);
        if (lx < 0 || lx >= W * mw || ly < 0 || ly >= H * mh) return nullptr;
        const int npy = ly / (2 * mh), r = ly % (2 * mh);
        const MbState& top = D.mbs_[(size_t)(2 * npy) * W + lx / mw];
        const bool nf = top.slice_nr == slice_nr && top.fld;
        const int nb = nf ? (ly & 1) : (r >= mh);
        ax = lx;
        ay = npy * 2 * mh + (nf ? r / 2 + (ly & 1) * mh : r);
        MbState* m = &D.mbs_[(size_t)(2 * npy + nb) * W + lx / mw];
        return m->slice_nr == slice_nr ? m : nullptr;
    }
    ax = mbx * mw + xN;
    ay = mby * mh + yN;
    if (ax < 0 || ax >= W * mw || ay < 0 || ay >= H * mh) return nullptr;
    MbState* m = &D.mbs_[(size_t)(ay / mh) * W + ax / mw];
    return m->slice_nr == slice_nr ? m : nullptr;
}

void SliceCtx::macroblock()
{
    si = mbaff ? ((addr >> 1) / W * 2 + (addr & 1)) * W + (addr >> 1) % W : addr;
    mbx = si % W;
    mby = si / W;
    MbState& m = D.mbs_[si];
    cur = &m;
    // macroblock_t::init (slice_data.cc:455-524)
    m.slice_nr = slice_nr;
    chroma_mode = 0;
    cbpl = cbpc = 0;
    cbp_blks = 0;
    m.cbp_bits = 0;
    if (sh.slice_type != H264R_SLICE_I) memset(m.mvd, 0, sizeof(m.mvd));
    memset(cof, 0, sizeof(cof));
    allrefzero = false;
    const bool I = sh.slice_type == H264R_SLICE_I, B = sh.slice_type == H264R_SLICE_B;
    int mb_type;
    skip = false;
    const bool top = (addr & 1) == 0, prev_skipped = mbaff && !top && D.mbs_[si - W].skip;
    if (mbaff) {
        // mb_field_decoding_flag, inferred first (macroblock_t::init slice_data.cc:505-523): a pair's top
        // MB, or a bottom MB whose top MB was skipped, takes the flag of the pair to the left (its top MB),
        // else of the pair above (its bottom MB), in the slice, else frame; a bottom MB after a coded top
        // MB takes the top MB's.  The CABAC skip contexts see the inferred flag.
        if (top || prev_skipped) {
            const int py = mby >> 1;
            const MbState* A = mbx > 0 ? &D.mbs_[(size_t)(2 * py) * W + mbx - 1] : nullptr;
            const MbState* Bm = py > 0 ? &D.mbs_[(size_t)(2 * py - 1) * W + mbx] : nullptr;
            if (A && A->slice_nr == slice_nr) m.fld = A->fld;
            else if (Bm && Bm->slice_nr == slice_nr) m.fld = Bm->fld;
            else m.fld = false;
        } else
            m.fld = D.mbs_[si - W].fld;
    } else
        m.fld = false;
    if (!I) {
        if (cab) {
            // mb_skip_flag: ctxIdxInc = A / B available and not skipped
            if (pre_skip_read) {
                pre_skip_read = false;
                skip = pre_skip;
            } else {
                int inc = 0;
                for (MbState* n : {nb_cur(-1, 0), nb_cur(0, -1)}) inc += n && !n->skip;
                skip = cab->dec(CTX_SKIP_CONTEXTS + inc);
                if (skip) last_dquant = 0;
            }
        } else {
            if (skip_run == -1) skip_run = b.ue_max(W * H, "mb_skip_run");
            skip = skip_run > 0;
            run_now = skip_run;
            --skip_run;
        }
    }
    m.skip = skip;
    if (mbaff) {
        // the coded flag: CAVLC -- a skipped top MB whose skip run ends with it takes the bottom MB's
        // (a peek, interpret_mb.cc:233-236); CABAC -- a skipped top MB reads the bottom MB's skip flag
        // ahead, with the bottom MB taking the top MB's inferred flag, and then, when the bottom MB is
        // coded, the pair's flag (:210-231).  A coded MB reads it when it is a top MB or follows a
        // skipped top MB (:250-262).
        if (cab) {
            if (top && skip) {
                MbState& bm = D.mbs_[si + W];
                bm.slice_nr = slice_nr;
                bm.fld = m.fld;
                cur = &bm;
                ++mby;
                int inc = 0;
                for (MbState* n : {nb_cur(-1, 0), nb_cur(0, -1)}) inc += n && !n->skip;
                pre_skip = cab->dec(CTX_SKIP_CONTEXTS + inc);
                pre_skip_read = true;
                if (!pre_skip) {
                    pre_fld = cabac_field_flag() != 0;
                    pre_fld_read = true;
                    m.fld = pre_fld;
                }
                cur = &m;
                --mby;
            }
            if (!skip && (top || prev_skipped)) {
                if (pre_fld_read) { pre_fld_read = false; m.fld = pre_fld; }
                else m.fld = cabac_field_flag() != 0;
            }
        } else {
            if (top && skip && run_now == 1) m.fld = b.peek(1) != 0;
            if (!skip && (top || prev_skipped)) m.fld = b.u(1) != 0;
        }
        zz4 = m.fld ? FIELD_SCAN4X4 : ZZ4;                   // a field MB's scans (transform.cc:344-357)
        zz8 = m.fld ? FIELD_SCAN8X8 : ZZ8;
    }
    mb_type = skip ? 0 : (cab ? cabac_mb_type(I, B) : b.ue_max(48, "mb_type")) + ((!I && !B) ? 1 : 0);
    // mb_type tables (interpret_mb.cc:318-406)
    int itype = -1;
    if (I) itype = mb_type;
    else if (!B) { if (mb_type >= 6) itype = mb_type - 6; }
    else if (mb_type >= 23) itype = mb_type - 23;
    int pred_a = 0, pred_b = 0;   // B partition prediction modes
    if (itype >= 0) {
        require(itype <= 25, "mb_type");
        m.intra = true;
        if (itype == 0) { m.mb_type = H264R_I_4x4; m.i16 = 0; }
        else if (itype == 25) { m.mb_type = H264R_I_PCM; m.i16 = 0; }
        else {
            m.mb_type = H264R_I_16x16;
            m.i16 = (uint8_t)((itype - 1) % 4);
            cbpc = ((itype - 1) / 4) % 3;
            cbpl = itype >= 13 ? 15 : 0;
        }
    } else if (!B) {
        require(mb_type <= 5, "mb_type (P)");
        m.intra = false;
        if (mb_type == 0) {
            m.mb_type = 0;
            memset(m.sub_type, 0, 4);
            memset(m.sub_pred, 0, 4);
        } else {
            static const uint8_t T[5] = {1, 2, 3, 4, 4};
            m.mb_type = T[mb_type - 1];
            allrefzero = mb_type == 5;
            memset(m.sub_type, m.mb_type, 4);
            memset(m.sub_pred, 0, 4);
        }
    } else {
        require(mb_type <= 22, "mb_type (B)");
        // Table 7-14 (interpret_mb.cc:83-109): {type, pred of partition 0, of partition 1}
        static const uint8_t T[23][3] = {
            {0, 2, 0}, {1, 0, 0}, {1, 1, 0}, {1, 2, 0}, {2, 0, 0}, {3, 0, 0}, {2, 1, 1}, {3, 1, 1},
            {2, 0, 1}, {3, 0, 1}, {2, 1, 0}, {3, 1, 0}, {2, 0, 2}, {3, 0, 2}, {2, 1, 2}, {3, 1, 2},
            {2, 2, 0}, {3, 2, 0}, {2, 2, 1}, {3, 2, 1}, {2, 2, 2}, {3, 2, 2}, {4, 0, 0}};
        m.intra = false;
        m.mb_type = T[mb_type][0];
        pred_a = T[mb_type][1];
        pred_b = T[mb_type][2];
        memset(m.sub_type, m.mb_type, 4);
        for (int i = 0; i < 4; ++i)
            m.sub_pred[i] = m.mb_type == 1 ? pred_a : m.mb_type == 2 ? (i / 2 ? pred_b : pred_a) : (i % 2 ? pred_b : pred_a);
        if (m.mb_type == 2 && pred_a == 2 && pred_b == 2) {}   // (table values as above)
    }
    if (skip) { cbpl = 0; cbpc = 0; }

    if (m.mb_type == H264R_I_PCM) {
        // parse_i_pcm (interpret_mb.cc:408-478)
        m.t8 = false;
        update_qp(0);
        memset(m.nz, 16, sizeof(m.nz));
        cbp_blks = 0xFFFF;
        reset_motion();
        m.skip = false;
        last_dquant = 0;
        m.cbpl = m.cbpc = 0;
        m.cmode = 0;
        while (!b.aligned()) b.u(1);
        for (int y = 0; y < 16; ++y)
            for (int x = 0; x < 16; ++x) cof[0][y][x] = b.u(8);
        for (int c = 1; c <= 2; ++c)
            for (int y = 0; y < mhc; ++y)
                for (int x = 0; x < mwc; ++x) cof[c][y][x] = b.u(8);
        if (cab) cab->init_engine(b);
        stage();
        return;
    }
    // sub_mb_type (interpret_mb.cc:480-503)
    if (!m.intra) {
        no_sub_lt8 = true;
        m.t8 = false;
        if (m.mb_type == H264R_P_8x8) {
            for (int k = 0; k < 4; ++k) {
                const uint32_t t = cab ? (uint32_t)cabac_sub_mb_type(B) : b.ue();
                if (!B) {
                    require(t < 4, "sub_mb_type (P)");
                    m.sub_type[k] = (uint8_t)(4 + t);        // P_8x8, P_8x4, P_4x8, P_4x4
                    m.sub_pred[k] = 0;
                } else {
                    require(t < 13, "sub_mb_type (B)");
                    // Table 7-18: {type, pred}
                    static const uint8_t S[13][2] = {{0, 2}, {4, 0}, {4, 1}, {4, 2}, {5, 0}, {6, 0}, {5, 1},
                                                     {6, 1}, {5, 2}, {6, 2}, {7, 0}, {7, 1}, {7, 2}};
                    m.sub_type[k] = S[t][0];
                    m.sub_pred[k] = S[t][1];
                }
                no_sub_lt8 &= m.sub_type[k] == 4 || (m.sub_type[k] == 0 && sps.direct_8x8_inference);
            }
        }
    }
    if (m.intra) intra_pred_modes();
    else inter_pred();
    update_qp(qp);
    if (m.mb_type == 0) {
        m.t8 = false;
        if (sh.slice_type != H264R_SLICE_B) { set_cbp_state(); stage(); return; }   // P_Skip (nz cleared by skip_p)
        if (skip) {                                                                 // B_Skip
            memset(m.nz, 0, sizeof(m.nz));
            set_cbp_state();
            stage();
            return;
        }
    }
    // coded_block_pattern (interpret_mb.cc:707-729)
    if (m.mb_type != H264R_I_16x16) {
        int cbp;
        if (cab) {
            cbp = cabac_cbp();
            if (!cbp) last_dquant = 0;
        } else {
            if (cf == 0 || cf == 3) {      // Table 9-4, ChromaArrayType 0 / 3: no chroma CBP
                const int code = b.ue_max(15, "coded_block_pattern");
                cbp = m.intra ? CBP_ME_INTRA_444[code] : CBP_ME_INTER_444[code];
            } else {
                const int code = b.ue_max(47, "coded_block_pattern");
                cbp = m.intra ? CBP_ME_INTRA[code] : CBP_ME_INTER[code];
            }
        }
        cbpl = cbp % 16;
        cbpc = cbp / 16;
        const bool direct = m.mb_type == 0 && B;
        if (cbpl > 0 && pps.transform_8x8 && !m.intra && no_sub_lt8 && (!direct || sps.direct_8x8_inference))
            m.t8 = read_t8();
    }
    set_cbp_state();
    if (cbpl > 0 || cbpc > 0 || m.mb_type == H264R_I_16x16) {
        int dq;
        if (cab) {
            // unary at {last_dquant != 0, 2, 3}, mapped to the signed value (interpret_se.cc:441-460)
            const int inc[3] = {last_dquant != 0 ? 1 : 0, 2, 3};
            const int v = cab->unary(CTX_DELTA_QP_CONTEXTS, inc, 3);
            dq = (int8_t)((v & 1) ? (v + 1) >> 1 : -((v + 1) >> 1));
            last_dquant = dq;
        } else
            dq = b.se_in(-26, 25, "mb_qp_delta");
        require(dq >= -26 && dq <= 25, "mb_qp_delta");
        qp = (qp + dq + 52) % 52;
    }
    update_qp(qp);
    residual();
    stage();
}

// transform_size_8x8_flag: ctxIdxInc = A / B available with the 8x8 transform
bool SliceCtx::read_t8()
{
    if (!cab) return b.u(1);
    int inc = 0;
    for (MbState* n : {nb_cur(-1, 0), nb_cur(0, -1)}) inc += n && n->t8;
    return cab->dec(CTX_TRANSFORM_SIZE_CONTEXTS + inc);
}

void SliceCtx::set_cbp_state()
{
    cur->cbpl = (uint8_t)cbpl;
    cur->cbpc = (uint8_t)cbpc;
    cur->cmode = chroma_mode;
}

// mb_pred for intra MBs (interpret_mb.cc:506-569)
void SliceCtx::intra_pred_modes()
{
    MbState& m = *cur;
    reset_motion();
    m.t8 = false;
    if (pps.transform_8x8 && m.mb_type == H264R_I_4x4) {
        m.t8 = read_t8();
        m.mb_type = m.t8 ? H264R_I_8x8 : H264R_I_4x4;
    }
    // prev_intra_pred_mode_flag + rem_intra_pred_mode (interpret_se.cc:302-323: CABAC rem as 3
    // bins, LSB first, at ipr_contexts[1])
    auto read_mode = [&](bool& prev) -> int {
        if (!cab) {
            prev = b.u(1);
            return prev ? 0 : (int)b.u(3);
        }
        prev = cab->dec(CTX_IPR_CONTEXTS);
        if (prev) return 0;
        int r = 0;
        for (int k = 0; k < 3; ++k) r |= cab->dec(CTX_IPR_CONTEXTS + 1) << k;
        return r;
    };
    if (m.mb_type == H264R_I_4x4) {
        for (int k = 0; k < 16; ++k) {
            const int bx = ((k / 4) % 2) * 8 + ((k % 4) % 2) * 4, by = ((k / 4) / 2) * 8 + ((k % 4) / 2) * 4;
            bool prev;
            const int rem = read_mode(prev);
            const int pred = pred_mode(bx, by, false);
            m.i4[k] = (uint8_t)(prev ? pred : rem < pred ? rem : rem + 1);
        }
    } else if (m.mb_type == H264R_I_8x8) {
        for (int k = 0; k < 4; ++k) {
            bool prev;
            const int rem = read_mode(prev);
            const int pred = pred_mode((k % 2) * 8, (k / 2) * 8, true);
            m.i8[k] = (uint8_t)(prev ? pred : rem < pred ? rem : rem + 1);
        }
    }
    if (cf == 0 || cf == 3) {
        // no intra_chroma_pred_mode in 4:0:0 / 4:4:4 (7.3.5.1: ChromaArrayType 1 or 2)
    } else if (cab) {
        // TU cMax 3: bin 0 at A / B available with a non-DC chroma mode (not I_PCM), then 3
        int inc0 = 0;
        for (MbState* n : {nb_cur(-1, 0), nb_cur(0, -1)}) inc0 += n && n->cmode != 0 && n->mb_type != H264R_I_PCM;
        const int inc[2] = {inc0, 3};
        chroma_mode = (uint8_t)cab->tu(CTX_CIPR_CONTEXTS, inc, 2, 3);
    } else
        chroma_mode = (uint8_t)b.ue_max(3, "intra_chroma_pred_mode");
    require(chroma_mode <= 3, "intra_chroma_pred_mode");
}

// predIntra4x4PredMode / predIntra8x8PredMode (neighbour.cc:318-397)
uint8_t SliceCtx::pred_mode(int bx, int by, bool n8)
{
    static const int scan[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
    int ax, ay, bxx, byy;
    MbState* A = nb_mb(false, bx - 1, by, ax, ay);
    MbState* Bm = nb_mb(false, bx, by - 1, bxx, byy);
    if (pps.cip) {
        if (A && !A->intra) A = nullptr;
        if (Bm && !Bm->intra) Bm = nullptr;
    }
    if (!A || !Bm) return 2;
    auto mode = [&](MbState* n, int x, int y) -> int {
        const int k = scan[(y & 12) + (x & 15) / 4];
        if (n->mb_type == H264R_I_8x8) return n->i8[k / 4];
        if (n->mb_type == H264R_I_4x4) return n->i4[k];
        return 2;
    };
    (void)n8;
    return (uint8_t)std::min(mode(A, ax, ay), mode(Bm, bxx, byy));
}

// both lists of the MB's 16 mv_info entries reset (interpret_mb.cc:508-519, 578-591)
void SliceCtx::reset_motion()
{
    Motion& M = *D.mot_;
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            const size_t i = M.at(mbx * 4 + x, mby * 4 + y);
            for (int l = 0; l < 2; ++l) {
                M.ref_idx[l][i] = -1;
                M.mvx[l][i] = M.mvy[l][i] = 0;
                M.ref_pic[l][i] = -1;
            }
        }
}

// neighbour_mv (interpret_mv.cc:27-114): A, B, C (or D) of the block at 4x4 position (i, j)
// of width w / height h (samples)
void SliceCtx::neighbour_mv(int list, int i, int j, int w, int h, bool avail[3], int ref[3], int mv[3][2])
{
    (void)h;
    int xa, ya, xb, yb, xc, yc, xd, yd;
    MbState* A = nb_mb(false, i * 4 - 1, j * 4, xa, ya);
    MbState* Bm = nb_mb(false, i * 4, j * 4 - 1, xb, yb);
    MbState* Cm = nb_mb(false, i * 4 + w, j * 4 - 1, xc, yc);
    MbState* Dm = nb_mb(false, i * 4 - 1, j * 4 - 1, xd, yd);
    if (j > 0) {
        if (i < 2) {
            if (j == 2) { if (w == 16) Cm = nullptr; }
            else if (i * 4 + w == 8) Cm = nullptr;
        } else if (i * 4 + w == 16) Cm = nullptr;
    }
    if (!Cm) { Cm = Dm; xc = xd; yc = yd; }
    const Motion& M = *D.mot_;
    MbState* N[3] = {A, Bm, Cm};
    const int X[3] = {xa, xb, xc}, Y[3] = {ya, yb, yc};
    for (int k = 0; k < 3; ++k) {
        avail[k] = N[k] != nullptr;
        ref[k] = -1;
        mv[k][0] = mv[k][1] = 0;
        if (N[k] && !N[k]->intra) {
            const size_t e = M.at(X[k] / 4, Y[k] / 4);
            ref[k] = M.ref_idx[list][e];
            mv[k][0] = M.mvx[list][e];
            mv[k][1] = M.mvy[list][e];
            if (mbaff && cur->fld && !N[k]->fld) {         // interpret_mv.cc:60-104: field MB, frame neighbour
                if (ref[k] >= 0) ref[k] *= 2;
                mv[k][1] /= 2;
            } else if (mbaff && !cur->fld && N[k]->fld) {  // frame MB, field neighbour
                ref[k] >>= 1;
                mv[k][1] *= 2;
            }
        }
    }
}

// predict_mv (interpret_mv.cc:116-149)
void SliceCtx::predict_mv(const bool avail[3], const int ref[3], const int mv[3][2], int r, int i, int j, int w, int h,
                          int out[2])
{
    const int* m;
    if (w == 8 && h == 16 && i == 0 && ref[0] == r) m = mv[0];
    else if (w == 8 && h == 16 && i != 0 && ref[2] == r) m = mv[2];
    else if (w == 16 && h == 8 && j == 0 && ref[1] == r) m = mv[1];
    else if (w == 16 && h == 8 && j != 0 && ref[0] == r) m = mv[0];
    else if (avail[0] && !avail[1] && !avail[2]) m = mv[0];
    else if (ref[0] == r && ref[1] != r && ref[2] != r) m = mv[0];
    else if (ref[0] != r && ref[1] == r && ref[2] != r) m = mv[1];
    else if (ref[0] != r && ref[1] != r && ref[2] == r) m = mv[2];
    else {
        out[0] = median(mv[0][0], mv[1][0], mv[2][0]);
        out[1] = median(mv[0][1], mv[1][1], mv[2][1]);
        return;
    }
    out[0] = m[0];
    out[1] = m[1];
}

// P_Skip (interpret_mv.cc:158-190)
void SliceCtx::skip_p()
{
    bool av[3];
    int ref[3], mv[3][2];
    neighbour_mv(0, 0, 0, 16, 16, av, ref, mv);
    int p[2] = {0, 0};
    if (!(!av[0] || (ref[0] == 0 && mv[0][0] == 0 && mv[0][1] == 0) || !av[1] ||
          (ref[1] == 0 && mv[1][0] == 0 && mv[1][1] == 0)))
        predict_mv(av, ref, mv, 0, 0, 0, 16, 16, p);
    Motion& M = *D.mot_;
    const int pic = list_[0][0] ? list_[0][0]->id : -1;
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            const size_t i = M.at(mbx * 4 + x, mby * 4 + y);
            M.ref_pic[0][i] = pic;
            M.ref_idx[0][i] = 0;
            M.mvx[0][i] = (int16_t)p[0];
            M.mvy[0][i] = (int16_t)p[1];
        }
    cbpl = cbpc = 0;
    memset(cur->nz, 0, sizeof(cur->nz));
}

static int rsd(int x) { return (x & 2) ? (x | 1) : (x & ~1); }

// get_colocated (interpret_mv.cc:192-240), frames and PAFF fields (direct_8x8_inference is 1
// whenever frame_mbs_only_flag is 0): the co-located 4x4 block of (i4, j4) in RefPicList1[0]'s
// motion -- a frame coded as frame: its own; a field of a frame coded as frame: the frame's
// rows 2 RSD(j4) (dpb_split_field picture.cc:541-569 copies them into both field views, and the
// reference takes the view of the CURRENT field's parity); a field of a frame coded as fields:
// that field's own; a frame coded as fields seen from a frame picture: the field nearer in POC,
// row RSD(j4) / 2
const Motion& SliceCtx::colocated(int i4, int j4, size_t& e)
{
    Picture* ref = list_[1][0];
    Picture* fs = ref->parent ? ref->parent : ref;
    const bool d8 = sps.direct_8x8_inference;
    if (sh.field) {
        if (!fs->fields) {
            require(fs->mot != nullptr, "co-located motion");
            e = fs->mot->at(rsd(i4), 2 * rsd(j4));
            return *fs->mot;
        }
        require(fs->mot_f[ref->parity] != nullptr, "co-located motion");
        const Motion& M = *fs->mot_f[ref->parity];
        e = M.at(rsd(i4), rsd(j4));
        return M;
    }
    if (fs->fields) {
        const int k = std::abs(D.cur_poc_ - fs->poc_f[1]) > std::abs(D.cur_poc_ - fs->poc_f[0]) ? 0 : 1;
        require(fs->mot_f[k] != nullptr, "co-located motion");
        e = fs->mot_f[k]->at(rsd(i4), rsd(j4) >> 1);
        return *fs->mot_f[k];
    }
    e = d8 ? fs->mot->at(rsd(i4), rsd(j4)) : fs->mot->at(i4, j4);
    return *fs->mot;
}

// get_direct_spatial (interpret_mv.cc:371-434), frames, direct_8x8_inference as signalled
void SliceCtx::direct_spatial()
{
    MbState& m = *cur;
    if (m.sub_type[0] && m.sub_type[1] && m.sub_type[2] && m.sub_type[3]) return;
    bool av0[3], av1[3];
    int r0[3], r1[3], mv0[3][2], mv1[3][2];
    neighbour_mv(0, 0, 0, 16, 16, av0, r0, mv0);
    neighbour_mv(1, 0, 0, 16, 16, av1, r1, mv1);
    auto min_pos = [](int a, int b, int c) {
        auto mp = [](int x, int y) { return (x >= 0 && y >= 0) ? std::min(x, y) : std::max(x, y); };
        return mp(a, mp(b, c));
    };
    int ref0 = min_pos(r0[0], r0[1], r0[2]), ref1 = min_pos(r1[0], r1[1], r1[2]);
    const bool zero = ref0 < 0 && ref1 < 0;
    if (zero) ref0 = ref1 = 0;
    int p0[2], p1[2];
    predict_mv(av0, r0, mv0, ref0, 0, 0, 16, 16, p0);
    predict_mv(av1, r1, mv1, ref1, 0, 0, 16, 16, p1);
    Motion& M = *D.mot_;
    Picture* col = list_[1][0];
    require(col != nullptr, "direct prediction without RefPicList1[0]");
    const int step = sps.direct_8x8_inference ? 4 : 1;
    for (int blk = 0; blk < 16; blk += step) {
        if (m.sub_type[blk / 4] != 0) continue;
        m.sub_pred[blk / 4] = ref1 < 0 ? 0 : ref0 < 0 ? 1 : 2;
        const int i = ((blk / 4) % 2) * 2 + ((blk % 4) % 2), j = ((blk / 4) / 2) * 2 + ((blk % 4) / 2);
        bool colzero = false;
        if (!col->long_term) {
            size_t e;
            const Motion& C = colocated(mbx * 4 + i, mby * 4 + j, e);
            colzero = (C.ref_idx[0][e] == 0 && std::abs(C.mvx[0][e]) >> 1 == 0 && std::abs(C.mvy[0][e]) >> 1 == 0) ||
                      (C.ref_idx[0][e] == -1 && C.ref_idx[1][e] == 0 && std::abs(C.mvx[1][e]) >> 1 == 0 &&
                       std::abs(C.mvy[1][e]) >> 1 == 0);
        }
        const size_t e = M.at(mbx * 4 + i, mby * 4 + j);
        M.ref_pic[0][e] = ref0 == -1 ? -1 : (list_[0][ref0] ? list_[0][ref0]->id : -1);
        M.ref_pic[1][e] = ref1 == -1 ? -1 : (list_[1][ref1] ? list_[1][ref1]->id : -1);
        M.ref_idx[0][e] = (int8_t)ref0;
        M.ref_idx[1][e] = (int8_t)ref1;
        const bool z0 = zero || ref0 < 0 || (ref0 == 0 && colzero), z1 = zero || ref1 < 0 || (ref1 == 0 && colzero);
        M.mvx[0][e] = (int16_t)(z0 ? 0 : p0[0]);
        M.mvy[0][e] = (int16_t)(z0 ? 0 : p0[1]);
        M.mvx[1][e] = (int16_t)(z1 ? 0 : p1[0]);
        M.mvy[1][e] = (int16_t)(z1 ? 0 : p1[1]);
        if (sps.direct_8x8_inference)
            for (int d = 1; d < 4; ++d) {
                const size_t f = M.at(mbx * 4 + i + (d & 1), mby * 4 + j + (d >> 1));
                for (int l = 0; l < 2; ++l) {
                    M.ref_pic[l][f] = M.ref_pic[l][e];
                    M.ref_idx[l][f] = M.ref_idx[l][e];
                    M.mvx[l][f] = M.mvx[l][e];
                    M.mvy[l][f] = M.mvy[l][e];
                }
            }
    }
}

// get_direct_temporal (interpret_mv.cc:192-369), frames
void SliceCtx::direct_temporal()
{
    MbState& m = *cur;
    if (m.sub_type[0] && m.sub_type[1] && m.sub_type[2] && m.sub_type[3]) return;
    Motion& M = *D.mot_;
    Picture* col = list_[1][0];
    require(col != nullptr, "direct prediction without RefPicList1[0]");
    unsupported(sh.field || col->fields || !col->mot, "temporal direct prediction with field pictures");
    const Motion& C = *col->mot;
    for (int blk = 0; blk < 16; ++blk) {
        if (m.sub_type[blk / 4] != 0) continue;
        m.sub_pred[blk / 4] = 2;
        const int i = ((blk / 4) % 2) * 2 + ((blk % 4) % 2), j = ((blk / 4) / 2) * 2 + ((blk % 4) / 2);
        const int i4 = mbx * 4 + i, j4 = mby * 4 + j;
        const size_t c = sps.direct_8x8_inference ? C.at(rsd(i4), rsd(j4)) : C.at(i4, j4);
        const int rl = C.ref_idx[0][c] == -1 ? 1 : 0;
        const int ridx = C.ref_idx[rl][c];
        const size_t e = M.at(i4, j4);
        if (ridx == -1) {
            M.ref_idx[0][e] = 0;
            M.mvx[0][e] = M.mvy[0][e] = 0;
            M.mvx[1][e] = M.mvy[1][e] = 0;
        } else {
            const int mvc[2] = {C.mvx[rl][c], C.mvy[rl][c]};
            // MapColToList0 (:242-285): the list-0 index of the picture the co-located block used
            const int cpic = C.ref_pic[rl][c];
            int mapped = -1;
            const int nref = std::min(sh.nref[0], list_n_[0]);
            for (int k = 0; k < nref; ++k)
                if (list_[0][k] && list_[0][k]->id == cpic) { mapped = k; break; }
            require(mapped >= 0, "temporal direct: co-located block's reference is unavailable");
            // DistScaleFactor (:287-311)
            const Picture* p0 = list_[0][mapped];
            const Picture* p1 = list_[1][0];
            int scale = 9999;
            if (!p0->long_term) {
                const int tb = clip3(-128, 127, D.cur_poc_ - p0->poc), td = clip3(-128, 127, p1->poc - p0->poc);
                if (td != 0) {
                    const int tx = (16384 + std::abs(td / 2)) / td;
                    scale = clip3(-1024, 1023, (tb * tx + 32) >> 6);
                }
            }
            M.ref_idx[0][e] = (int8_t)mapped;
            if (scale == 9999) {
                M.mvx[0][e] = (int16_t)mvc[0];
                M.mvy[0][e] = (int16_t)mvc[1];
                M.mvx[1][e] = M.mvy[1][e] = 0;
            } else {
                M.mvx[0][e] = (int16_t)((scale * mvc[0] + 128) >> 8);
                M.mvy[0][e] = (int16_t)((scale * mvc[1] + 128) >> 8);
                M.mvx[1][e] = (int16_t)(M.mvx[0][e] - mvc[0]);
                M.mvy[1][e] = (int16_t)(M.mvy[0][e] - mvc[1]);
            }
        }
        M.ref_idx[1][e] = 0;
        M.ref_pic[0][e] = list_[0][M.ref_idx[0][e]] ? list_[0][M.ref_idx[0][e]]->id : -1;
        M.ref_pic[1][e] = list_[1][0] ? list_[1][0]->id : -1;
    }
}

// mb_pred for inter MBs (interpret_mb.cc:571-705, interpret_mv.cc:151-190)
void SliceCtx::inter_pred()
{
    MbState& m = *cur;
    const bool B = sh.slice_type == H264R_SLICE_B;
    if (!B && m.mb_type == 0) { skip_p(); return; }
    if (m.mb_type != 0) reset_motion();
    if (B && (m.mb_type == 0 || m.mb_type == H264R_P_8x8)) {
        if (sh.direct_spatial) direct_spatial();
        else direct_temporal();
    }
    if (B && m.mb_type == 0) return;
    static const int STEP[8][2] = {{0, 0}, {4, 4}, {4, 2}, {2, 4}, {2, 2}, {2, 1}, {1, 2}, {1, 1}};
    Motion& M = *D.mot_;
    const int sh0 = STEP[m.mb_type][0], sv0 = STEP[m.mb_type][1];
    const int nlists = B ? 2 : 1;
    // ref_idx_l0 / ref_idx_l1 (interpret_mb.cc:632-658; interpret_se.cc:341-370)
    for (int l = 0; l < nlists; ++l)
        for (int y8 = 0; y8 < 4; y8 += sv0)
            for (int x8 = 0; x8 < 4; x8 += sh0) {
                const int part = 2 * (y8 >> 1) + (x8 >> 1);
                if ((m.sub_pred[part] == l || m.sub_pred[part] == 2) && m.sub_type[part] != 0) {
                    const bool present = B || !allrefzero || m.mb_type != H264R_P_8x8;
                    // te() range: a field MB's refIdx counts fields (the reference doubles num_ref_idx_active
                    // for the MB, interpret_mb.cc:271-275, and halves it after, slice_data.cc:648-651)
                    const int n = sh.nref[l] * (m.fld ? 2 : 1);
                    int r = 0;
                    if (present && n > 1) r = cab ? cabac_ref_idx(l, x8, y8) : n == 2 ? 1 - (int)b.u(1) : b.ue_max(63, "ref_idx");
                    require(r >= 0 && r < sh.nref[l] * (m.fld ? 2 : 1), "ref_idx out of range");
                    for (int y4 = 0; y4 < sv0; ++y4)
                        for (int x4 = 0; x4 < sh0; ++x4) M.ref_idx[l][M.at(mbx * 4 + x8 + x4, mby * 4 + y8 + y4)] = (int8_t)r;
                }
            }
    // mvd_l0 / mvd_l1 (:660-705)
    for (int l = 0; l < nlists; ++l)
        for (int y8 = 0; y8 < 4; y8 += sv0)
            for (int x8 = 0; x8 < 4; x8 += sh0) {
                const int part = 2 * (y8 >> 1) + (x8 >> 1);
                if (!((m.sub_pred[part] == l || m.sub_pred[part] == 2) && m.sub_type[part] != 0)) continue;
                const int sh4 = STEP[m.sub_type[part]][0], sv4 = STEP[m.sub_type[part]][1];
                const int cref = M.ref_idx[l][M.at(mbx * 4 + x8, mby * 4 + y8)];
                for (int y4 = 0; y4 < sv0; y4 += sv4)
                    for (int x4 = 0; x4 < sh0; x4 += sh4) {
                        const int dx = (int16_t)(cab ? cabac_mvd(l, x8 + x4, y8 + y4, 0) : b.se());
                        const int dy = (int16_t)(cab ? cabac_mvd(l, x8 + x4, y8 + y4, 1) : b.se());
                        bool av[3];
                        int ref[3], mv[3][2], p[2];
                        neighbour_mv(l, x8 + x4, y8 + y4, sh4 * 4, sv4 * 4, av, ref, mv);
                        predict_mv(av, ref, mv, cref, x8 + x4, y8 + y4, sh4 * 4, sv4 * 4, p);
                        const int16_t vx = (int16_t)(dx + p[0]), vy = (int16_t)(dy + p[1]);
                        for (int y2 = 0; y2 < sv4; ++y2)
                            for (int x2 = 0; x2 < sh4; ++x2) {
                                const size_t e = M.at(mbx * 4 + x8 + x4 + x2, mby * 4 + y8 + y4 + y2);
                                M.mvx[l][e] = vx;
                                M.mvy[l][e] = vy;
                                int16_t* d = m.mvd[l][(y8 + y4 + y2) * 4 + x8 + x4 + x2];
                                d[0] = (int16_t)dx;
                                d[1] = (int16_t)dy;
                            }
                    }
            }
    // reference picture ids for deblocking (:611-623)
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            const size_t e = M.at(mbx * 4 + x, mby * 4 + y);
            for (int l = 0; l < nlists; ++l) {
                // an MBAFF field MB's refIdx r names a field of frame r / 2 (get_ref_pic dpb.cc:1046-1055)
                const int r = m.fld && M.ref_idx[l][e] >= 0 ? M.ref_idx[l][e] >> 1 : M.ref_idx[l][e];
                M.ref_pic[l][e] = (r >= 0 && list_[l][r]) ? list_[l][r]->id : -1;
            }
        }
}

// predict_nnz (neighbour.cc:263-314): nC of the 4x4 block at sample (i, j) of plane pl
int SliceCtx::nnz_pred(int pl, int i, int j)
{
    const bool chroma = pl != 0 && cf != 3;                 // 4:4:4: Cb / Cr blocks in the luma grid
    const int mw = chroma ? 8 : 16, mh = chroma ? mhc : 16;
    int xa, ya, xb, yb;
    MbState* A = nb_mb(chroma, i - 1, j, xa, ya);
    MbState* Bm = nb_mb(chroma, i, j - 1, xb, yb);
    int nA = A ? A->nz[pl][(ya % mh) / 4][(xa % mw) / 4] : 0;
    int nB = Bm ? Bm->nz[pl][(yb % mh) / 4][(xb % mw) / 4] : 0;
    int nC = nA + nB;
    if (A && Bm) nC = (nC + 1) >> 1;
    return nC;
}

// residual_block_cavlc (interpret_residual.cc:64-174): the coefficients as (scan position,
// level) pairs; returns TotalCoeff.  blk = blkIdx (luma) or the chroma 4x4 index.
int SliceCtx::block_cavlc(int pl, bool chroma, bool ac, int blk, int start, int max_coeff, int32_t* out, int* nout)
{
    const Tables& T = tables();
    const int i = chroma ? blk % 2 : ((blk / 4) % 2) * 2 + (blk % 4) % 2;
    const int j = chroma ? blk / 2 : ((blk / 4) / 2) * 2 + (blk % 4) / 2;
    int nC = (chroma && !ac) ? (cf == 2 ? -2 : -1) : nnz_pred(pl, i * 4, j * 4);
    int tc, t1;
    if (nC >= 8) {
        const int c = b.u(6);
        if (c == 3) tc = t1 = 0;
        else { tc = (c >> 2) + 1; t1 = c & 3; }
    } else {
        const int cls = nC == -1 ? 3 : nC == -2 ? 4 : nC < 2 ? 0 : nC < 4 ? 1 : 2;
        const int v = T.coeff_token[cls].read(b, "coeff_token");
        tc = v >> 2;
        t1 = v & 3;
    }
    require(tc <= max_coeff, "coeff_token: TotalCoeff above the block size");
    require(t1 <= tc, "coeff_token: TrailingOnes above TotalCoeff");       // the 6-bit FLC (nC >= 8) can say so
    int level[16], run[16];
    if (tc > 0) {
        int suffix = tc > 10 && t1 < 3 ? 1 : 0;
        if (t1) {
            const int code = b.u(t1);
            int ntr = t1;
            for (int k = tc - 1; k > tc - 1 - t1; --k) level[k] = 1 - 2 * ((code >> (--ntr)) & 1);
        }
        for (int k = tc - 1 - t1; k >= 0; --k) {
            int prefix = -1;
            for (int bit = 0; !bit; ++prefix) {
                bit = b.bit();
                if (prefix > 32) fail(H264R_EINVAL, "level_prefix too long");
            }
            const int ssize = (prefix == 14 && suffix == 0) ? 4 : prefix >= 15 ? prefix - 3 : suffix;
            const int lsuf = ssize > 0 ? (int)b.u(ssize) : 0;
            int code = (std::min(15, prefix) << suffix) + lsuf;
            if (prefix >= 15 && suffix == 0) code += 15;
            if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
            if (k == tc - 1 - t1 && t1 < 3) code += 2;
            level[k] = (code % 2) == 0 ? (code + 2) >> 1 : (-code - 1) >> 1;
            if (suffix == 0) suffix = 1;
            if (std::abs(level[k]) > (3 << (suffix - 1)) && suffix < 6) ++suffix;
        }
        int zeros = 0;
        if (tc < max_coeff) {
            const int yuv = max_coeff == 4 ? 0 : max_coeff == 8 ? 1 : 2;
            zeros = T.total_zeros[yuv][tc].read(b, "total_zeros");
        }
        for (int k = tc - 1; k > 0; --k) {
            run[k] = zeros > 0 ? T.run_before[std::min(zeros, 7)].read(b, "run_before") : 0;
            zeros -= run[k];
        }
        run[0] = zeros;
        require(zeros >= 0, "run_before exceeds total_zeros");
    }
    if (ac) cur->nz[pl][j][i] = (uint8_t)tc;
    int num = start - 1, n = 0;
    for (int k = 0; k < tc; ++k) {
        num += run[k] + 1;
        require(num < start + max_coeff, "coefficient position past the block");
        out[2 * n] = num;
        out[2 * n + 1] = level[k];
        ++n;
    }
    *nout = n;
    return tc;
}

// residual_luma / residual_chroma (interpret_residual.cc:421-494) + the coefficient push
// of the shim (decoder_h264r.cc:328-354): raw levels at raster positions in cof
enum { LUMA_16DC, LUMA_16AC, LUMA_4x4, CHROMA_DC, CHROMA_AC, LUMA_8x8 };

void SliceCtx::residual()
{
    MbState& m = *cur;
    int32_t pl_[128];
    int n;
    const bool i16 = m.mb_type == H264R_I_16x16;
    // residual_luma for Y, and for Cb and Cr as luma in 4:4:4 (interpret_residual.cc:497-505);
    // cbp_blks is the luma plane's (the record's, deblock.cc:135,212)
    for (int p = 0; p < (cf == 3 ? 3 : 1); ++p) {
    const uint16_t bmask = p == 0 ? 0xFFFF : 0;                  // (4:0:0: the luma plane only)
    if (i16) {
        block(LUMA_16DC, p, false, false, 0, 0, 16, pl_, &n);
        for (int k = 0; k < n; ++k) {
            const int r = zz4[pl_[2 * k]];
            cof[p][(r / 4) * 4][(r % 4) * 4] = pl_[2 * k + 1];
        }
    }
    for (int i8 = 0; i8 < 4; ++i8) {
        if (cab && m.t8) {
            // one 64-coefficient block per coded 8x8 (CABAC, :449-450)
            if (!(cbpl & (1 << i8))) continue;
            const int i = (i8 % 2) * 2, j = (i8 / 2) * 2;
            block(LUMA_8x8, p, false, true, i8 * 4, 0, 64, pl_, &n);
            for (int k = 0; k < n; ++k) {
                cbp_blks |= (uint16_t)(0x33u << (j * 4 + i)) & bmask;
                const int r = zz8[pl_[2 * k]];
                cof[p][j * 4 + r / 8][i * 4 + r % 8] = pl_[2 * k + 1];
            }
            continue;
        }
        for (int i4 = 0; i4 < 4; ++i4) {
            const int blk = i8 * 4 + i4;
            const int i = ((blk / 4) % 2) * 2 + (blk % 4) % 2, j = ((blk / 4) / 2) * 2 + (blk % 4) / 2;
            if (!(cbpl & (1 << i8))) { if (!cab) m.nz[p][j][i] = 0; continue; }
            if (i16) block(LUMA_16AC, p, false, true, blk, 1, 15, pl_, &n);
            else block(LUMA_4x4, p, false, true, blk, 0, 16, pl_, &n);
            for (int k = 0; k < n; ++k) {
                const int c = pl_[2 * k], lev = pl_[2 * k + 1];
                if (!m.t8) {
                    cbp_blks |= (uint16_t)(1u << (j * 4 + i)) & bmask;
                    const int r = zz4[c];
                    cof[p][j * 4 + r / 4][i * 4 + r % 4] = lev;
                } else {
                    // 8x8 CAVLC: four interleaved 4x4 readings (:161-164)
                    const int x0 = i & ~1, y0 = j & ~1;
                    cbp_blks |= (uint16_t)(0x33u << (y0 * 4 + x0)) & bmask;
                    const int r = zz8[c * 4 + blk % 4];
                    cof[p][y0 * 4 + r / 8][x0 * 4 + r % 8] = lev;
                }
            }
        }
    }
    }
    if (cf == 3 || cf == 0) return;
    // chroma: 4 (4:2:0) or 8 (4:2:2) 4x4 blocks and DC coefficients per plane; the 4:2:2 DC scan
    // (inverse_scan_chroma_dc transform.cc:365-374, the field 4x4 scan's first 8 positions) as
    // raster indices of the 2-wide DC matrix
    static const uint8_t DC422[8] = {0, 2, 1, 4, 6, 3, 5, 7};
    const int nbc = cf == 2 ? 8 : 4;
    if (cbpc & 3)
        for (int c = 1; c <= 2; ++c) {
            block(CHROMA_DC, c, true, false, 0, 0, nbc, pl_, &n);
            for (int k = 0; k < n; ++k) {
                const int q = cf == 2 ? DC422[pl_[2 * k]] : pl_[2 * k];
                cof[c][(q / 2) * 4][(q % 2) * 4] = pl_[2 * k + 1];
            }
        }
    for (int c = 1; c <= 2; ++c)
        for (int blk = 0; blk < nbc; ++blk) {
            if (!(cbpc & 2)) { if (!cab) m.nz[c][blk / 2][blk % 2] = 0; continue; }
            block(CHROMA_AC, c, true, true, blk, 1, 15, pl_, &n);
            for (int k = 0; k < n; ++k) {
                const int r = zz4[pl_[2 * k]];
                cof[c][(blk / 2) * 4 + r / 4][(blk % 2) * 4 + r % 4] = pl_[2 * k + 1];
            }
        }
}

// ------------------------------------------------------------------ CABAC syntax elements
// the MB at (dx, dy) MBs from the current one if it is in the current slice (get_mb + the
// slice_nr check of every CtxIdxInc function)
MbState* SliceCtx::nb_cur(int dx, int dy)
{
    int ax, ay;
    return nb_mb(false, dx * 16, dy * 16, ax, ay);
}

// mb_field_decoding_flag (interpret_se.cc:79-91, ctxIdxInc neighbour.cc:429-445): the pairs to the
// left and above, in the slice, coded as field pairs
int SliceCtx::cabac_field_flag()
{
    const int py = mby >> 1;
    const MbState* A = mbx > 0 ? &D.mbs_[(size_t)(2 * py) * W + mbx - 1] : nullptr;
    const MbState* Bm = py > 0 ? &D.mbs_[(size_t)(2 * py - 1) * W + mbx] : nullptr;
    const int inc = (A && A->slice_nr == slice_nr && A->fld) + (Bm && Bm->slice_nr == slice_nr && Bm->fld);
    return cab->dec(CTX_MB_AFF_CONTEXTS + inc);
}

// mb_type (interpret_se.cc:113-227): I-slice numbering 0..25 for I, P 0..3 (inter) / 5 + I,
// B 0..22 / 23 + I
int SliceCtx::cabac_mb_type(bool I, bool B)
{
    Cabac& c = *cab;
    auto i_suffix = [&](int base, bool islice) -> int {          // the I mb_type after the prefix bin
        if (c.term()) return 25;
        int t = 1;
        t += c.dec(base + (islice ? 3 : 1)) * 12;
        if (c.dec(base + (islice ? 4 : 2))) t += c.dec(base + (islice ? 5 : 2)) * 4 + 4;
        t += c.dec(base + (islice ? 6 : 3)) * 2;
        t += c.dec(base + (islice ? 7 : 3));
        return t;
    };
    if (I) {
        int inc = 0;
        for (MbState* n : {nb_cur(-1, 0), nb_cur(0, -1)}) inc += n && n->mb_type != H264R_I_4x4 && n->mb_type != H264R_I_8x8;
        const int base = CTX_MB_TYPE_CONTEXTS + 3;
        if (!c.dec(base + inc)) return 0;
        return i_suffix(base, true);
    }
    if (!B) {
        const int ctx = CTX_MB_TYPE_CONTEXTS;
        if (!c.dec(ctx + 0)) {
            if (!c.dec(ctx + 1)) return c.dec(ctx + 2) * 3;
            return 2 - c.dec(ctx + 3);
        }
        const int base = CTX_MB_TYPE_CONTEXTS + 3;
        if (!c.dec(base)) return 5;
        return 5 + i_suffix(base, false);
    }
    const int ctx = CTX_MB_TYPE_CONTEXTS;
    int inc = 0;
    for (MbState* n : {nb_cur(-1, 0), nb_cur(0, -1)}) inc += n && n->mb_type != 0;
    int t = 0;
    if (c.dec(ctx + inc)) {
        t = 1;
        if (!c.dec(ctx + 3)) t += c.dec(ctx + 5);
        else {
            t += 2;
            if (!c.dec(ctx + 4)) {
                t += c.dec(ctx + 5) * 4;
                t += c.dec(ctx + 5) * 2;
                t += c.dec(ctx + 5);
            } else {
                t += 9;
                t += c.dec(ctx + 5) * 8;
                t += c.dec(ctx + 5) * 4;
                t += c.dec(ctx + 5) * 2;
                if (t < 22) t += c.dec(ctx + 5);
                if (t == 22) t = 23;
                else if (t == 24) t = 11;
                else if (t == 26) t = 22;
            }
        }
    }
    if (t == 23) {
        const int base = CTX_MB_TYPE_CONTEXTS + 5;
        if (!c.dec(base)) return 23;
        return 23 + i_suffix(base, false);
    }
    return t;
}

// sub_mb_type (interpret_se.cc:247-285)
int SliceCtx::cabac_sub_mb_type(bool B)
{
    Cabac& c = *cab;
    const int ctx = CTX_B8_TYPE_CONTEXTS;
    int t = 0;
    if (!B) {
        if (!c.dec(ctx)) {
            t = 1;
            if (c.dec(ctx + 1)) t += c.dec(ctx + 2) ? 1 : 2;
        }
        return t;
    }
    if (c.dec(ctx)) {
        t = 1;
        if (c.dec(ctx + 1)) {
            t += 2;
            if (c.dec(ctx + 2)) {
                t += 4;
                if (c.dec(ctx + 3)) t += 4;
                else t += c.dec(ctx + 3) * 2;
            } else
                t += c.dec(ctx + 3) * 2;
        }
        t += c.dec(ctx + 3);
    }
    return t;
}

// coded_block_pattern (interpret_se.cc:419-435, neighbour.cc:635-686)
int SliceCtx::cabac_cbp()
{
    Cabac& c = *cab;
    int cbp = 0;
    MbState* A = nb_cur(-1, 0);
    MbState* Bm = nb_cur(0, -1);
    for (int y0 = 0; y0 < 4; y0 += 2)
        for (int x0 = 0; x0 < 4; x0 += 2) {
            int ca = 0x3F, cb = 0x3F, ia = 0, ib = 0;
            if (x0 == 0) {
                // the left 8x8 block holding the sample left of this one's top row (its row in MBAFF)
                int ax, ay;
                MbState* An = nb_mb(false, -1, y0 * 4, ax, ay);
                if (An && An->mb_type != H264R_I_PCM) { ca = An->cbpl; ia = ((((ay & 15) >> 2)) & ~1) + 1; }
            } else { ca = cbp; ia = y0; }
            if (y0 == 0) {
                if (Bm && Bm->mb_type != H264R_I_PCM) { cb = Bm->cbpl; ib = x0 / 2 + 2; }
            } else { cb = cbp; ib = x0 / 2; }
            const int inc = ((ca & (1 << ia)) == 0 ? 1 : 0) + 2 * ((cb & (1 << ib)) == 0 ? 1 : 0);
            if (c.dec(CTX_CBP_L_CONTEXTS + inc)) cbp += 1 << (y0 + (x0 >> 1));
        }
    if (cf == 0 || cf == 3) return cbp;                   // no chroma bins (interpret_se.cc:429)
    auto f = [](MbState* n, bool two) { return n && (n->mb_type == H264R_I_PCM || (two ? n->cbpc == 2 : n->cbpc != 0)); };
    const int inc0 = f(A, false) + 2 * f(Bm, false), inc1 = f(A, true) + 2 * f(Bm, true) + 4;
    if (c.dec(CTX_CBP_C_CONTEXTS + inc0)) cbp += c.dec(CTX_CBP_C_CONTEXTS + inc1) ? 32 : 16;
    return cbp;
}

// ref_idx_lX (interpret_se.cc:341-370, ctxIdxInc neighbour.cc:517-572): unary at {inc, 4, 5}
int SliceCtx::cabac_ref_idx(int list, int x4, int y4)
{
    const bool B = sh.slice_type == H264R_SLICE_B;
    const Motion& M = *D.mot_;
    int inc = 0;
    const int off[2][2] = {{x4 * 4 - 1, y4 * 4}, {x4 * 4, y4 * 4 - 1}};
    for (int k = 0; k < 2; ++k) {
        int ax, ay;
        MbState* n = nb_mb(false, off[k][0], off[k][1], ax, ay);
        if (!n) continue;
        const int r = M.ref_idx[list][M.at(ax / 4, ay / 4)];
        const int part = ((ay / 4) & 2) + ((ax / 8) & 1);
        const bool pred_eq = !((n->mb_type == 0 && B) || n->sub_type[part] == 0);
        // a frame MB over a field neighbour: refIdx > 1 (neighbour.cc:533-536)
        const bool zero = (mbaff && !cur->fld && n->fld) ? r <= 1 : r <= 0;
        const bool cond = !(n->mb_type == 0 || n->intra || !pred_eq || zero);
        inc += cond ? (k ? 2 : 1) : 0;
    }
    const int incs[3] = {inc, 4, 5};
    return cab->unary(CTX_REF_NO_CONTEXTS, incs, 3);
}

// mvd_lX (interpret_se.cc:372-387, ctxIdxInc neighbour.cc:574-633): UEG3, signed, cMax 9
int SliceCtx::cabac_mvd(int list, int x4, int y4, int comp)
{
    const bool B = sh.slice_type == H264R_SLICE_B;
    int sum = 0;
    const int off[2][2] = {{x4 * 4 - 1, y4 * 4}, {x4 * 4, y4 * 4 - 1}};
    for (int k = 0; k < 2; ++k) {
        int ax, ay;
        MbState* n = nb_mb(false, off[k][0], off[k][1], ax, ay);
        if (!n) continue;
        const int part = ((ay / 4) & 2) + ((ax / 8) & 1);
        const bool pred_eq = !((n->mb_type == 0 && B) || n->sub_type[part] == 0);
        if (!(n->mb_type == 0 || n->intra || !pred_eq)) {
            int v = std::abs((int)n->mvd[list][((ay & 15) / 4) * 4 + (ax & 15) / 4][comp]);
            if (mbaff && comp) {                          // vertical: field / frame units (neighbour.cc:599-604)
                if (!cur->fld && n->fld) v *= 2;
                else if (cur->fld && !n->fld) v /= 2;
            }
            sum += v;
        }
    }
    const int inc[5] = {sum < 3 ? 0 : sum <= 32 ? 1 : 2, 3, 4, 5, 6};
    return cab->ueg(comp ? CTX_MVD_Y_CONTEXTS : CTX_MVD_X_CONTEXTS, inc, 5, 9, 3, true);
}

// coded_block_flag ctxIdxInc (neighbour.cc:689-742)
int SliceCtx::cbf_inc(int pl, bool chroma, bool ac, int blk)
{
    const int i = chroma ? blk % 2 : ((blk / 4) % 2) * 2 + (blk % 4) % 2;
    const int j = chroma ? blk / 2 : ((blk / 4) / 2) * 2 + (blk % 4) / 2;
    const int bit = !chroma ? (ac ? 1 : 0) : !ac ? (pl == 1 ? 17 : 18) : (pl == 1 ? 19 : 35);
    const int nw = chroma ? mwc : 16, nh = chroma ? mhc : 16;     // MbWidthC / MbHeightC (neighbour.cc:716-722)
    int inc = 0;
    const int off[2][2] = {{i * 4 - 1, j * 4}, {i * 4, j * 4 - 1}};
    for (int k = 0; k < 2; ++k) {
        int ax, ay;
        MbState* n = nb_mb(chroma, off[k][0], off[k][1], ax, ay);
        int cond = cur->intra ? 1 : 0;
        if (n) {
            if (n->mb_type == H264R_I_PCM) cond = 1;
            else {
                const int pos = ac ? ((ay % nh) & 12) + (ax % nw) / 4 : 0;
                cond = (int)((n->cbp_bits >> (bit + pos)) & 1);
            }
        }
        inc += cond << k;
    }
    return inc;
}

// residual_block_cabac (interpret_residual.cc:315-419): (position, level) pairs, positions
// counted from 0 like the CAVLC reader's
int SliceCtx::block_cabac(int cat, int pl, bool chroma, bool ac, int blk, int start, int max_coeff, int32_t* out, int* nout)
{
    Cabac& c = *cab;
    *nout = 0;
    bool coded = true;                                    // always one for 8x8 blocks (4:2:0)
    if (cat != LUMA_8x8) coded = c.dec(CTX_BCBP_CONTEXTS + TYPE2CTX_BCBP[cat] + cbf_inc(pl, chroma, ac, blk));
    if (!coded) return 0;
    {                                                     // update_coded_block_flag (neighbour.cc:744-764)
        const int i = chroma ? blk % 2 : ((blk / 4) % 2) * 2 + (blk % 4) % 2;
        const int j = chroma ? blk / 2 : ((blk / 4) / 2) * 2 + (blk % 4) / 2;
        const int bit = (!chroma ? (ac ? 1 : 0) : !ac ? (pl == 1 ? 17 : 18) : (pl == 1 ? 19 : 35)) + (ac ? j * 4 + i : 0);
        cur->cbp_bits |= (uint64_t)(cur->t8 && !chroma && ac ? 0x33 : 0x01) << bit;
    }
    // field pictures: the second set of significance contexts and the field 8x8 map
    // (interpret_residual.cc:353-358)
    const bool fld = sh.field || cur->fld;                 // (field MBs of MBAFF frames too)
    // 4:2:2 chroma DC: CHROMA_DC_2x4's maps (ctxIdxInc Min(i / NumC8x8, 2); its context offsets are
    // CHROMA_DC's, interpret_residual.cc:336)
    const bool dc2x4 = cat == CHROMA_DC && cf == 2;
    const uint8_t* pmap = cat == LUMA_8x8 ? (fld ? POS2CTX_MAP8X8_FIELD : POS2CTX_MAP8X8) : dc2x4 ? POS2CTX_MAP2X4C : POS2CTX_MAP4X4;
    const uint8_t* plast = cat == LUMA_8x8 ? POS2CTX_LAST8X8 : dc2x4 ? POS2CTX_LAST2X4C : POS2CTX_LAST4X4;
    const int fset = fld ? (CTX_LAST_CONTEXTS - CTX_MAP_CONTEXTS) / 2 : 0;      // 210 contexts per set
    const int map = CTX_MAP_CONTEXTS + fset + TYPE2CTX_MAP[cat], last = CTX_LAST_CONTEXTS + fset + TYPE2CTX_MAP[cat];
    int sig[64];
    int num = max_coeff;
    int ii = 0;
    for (; ii < num - 1; ++ii) {
        sig[ii] = c.dec(map + pmap[ii]);
        if (sig[ii] && c.dec(last + plast[ii])) num = ii + 1;
    }
    sig[num - 1] = 1;
    const int one = CTX_ONE_CONTEXTS + TYPE2CTX_ONE[cat];
    int eq1 = 0, gt1 = 0, n = 0;
    for (int k = num - 1; k >= 0; --k) {
        if (!sig[k]) continue;
        const int inc0 = gt1 ? 0 : std::min(4, 1 + eq1);
        const int inc1 = 5 + std::min(4 - (cat == CHROMA_DC ? 1 : 0), gt1);
        int am1 = 0;
        if (c.dec(one + inc0)) {
            // unary_exp_golomb_level_decode (:291-312): up to 13 more bins at inc1, then EG0
            int ones = 0;
            while (ones < 13 && c.dec(one + inc1)) ++ones;
            if (ones < 13) am1 = ones + 1;
            else {
                int v = 0, kk = 0;
                while (c.bypass()) {
                    v += 1 << kk++;
                    if (kk > 24) fail(H264R_EINVAL, "CABAC: level suffix too long");
                }
                while (kk--) v += c.bypass() << kk;
                am1 = 14 + v;
            }
        }
        const int level = c.bypass() ? -(am1 + 1) : am1 + 1;
        out[2 * n] = k + start;
        out[2 * n + 1] = level;
        ++n;
        eq1 += am1 == 0;
        gt1 += am1 != 0;
    }
    *nout = n;
    return n;
}

// The MB's record, level block and motion as the shim's decode(mb) snapshots them
// (decoder_h264r.cc:364-468)
void SliceCtx::stage()
{
    MbState& m = *cur;
    if (sh.slice_type == H264R_SLICE_SP && !m.intra) {
        if (qsc[0] >= 6 || qsc[1] >= 6) fail(H264R_EUNSUPPORTED, "SP slice with QsC >= 6");
        if (m.t8) fail(H264R_EUNSUPPORTED, "8x8 transform in an SP slice");
        D.slice_tab_[slice_nr].qs_c[0] = (int8_t)qsc[0];
        D.slice_tab_[slice_nr].qs_c[1] = (int8_t)qsc[1];
    }
    StagedMb& st = D.staged_[si];
    h264r_mb& r = st.rec;
    memset(&r, 0, sizeof(r));
    r.mb_type = m.mb_type;
    r.flags = (uint8_t)((m.intra ? H264R_MBF_INTRA : 0) | (m.t8 ? H264R_MBF_T8x8 : 0) | (bypass ? H264R_MBF_BYPASS : 0) |
                        (m.fld ? H264R_MBF_FIELD : 0));
    r.cbp = (uint8_t)(cbpl | cbpc << 4);
    r.qp_y = (int8_t)qpy;
    r.qp_c[0] = (int8_t)qpc[0];
    r.qp_c[1] = (int8_t)qpc[1];
    r.i16_mode = m.i16;
    r.chroma_mode = chroma_mode;
    r.cbp_blks = cbp_blks;
    r.slice = (uint16_t)slice_nr;
    for (int k = 0; k < 3; ++k) r.qp_scaled[k] = (uint8_t)qp_scaled[k];
    const bool use8 = m.mb_type == H264R_I_8x8 || (bypass && !m.intra && m.t8);
    const bool use4 = m.mb_type == H264R_I_4x4 || (bypass && !m.intra && !m.t8);
    if (use8)
        for (int k = 0; k < 4; ++k) r.ipred[k >> 1] |= (uint8_t)((m.i8[k] & 15) << ((k & 1) * 4));
    else if (use4)
        for (int k = 0; k < 16; ++k) r.ipred[k >> 1] |= (uint8_t)((m.i4[k] & 15) << ((k & 1) * 4));
    std::vector<int16_t>& lv = st.levels;
    lv.clear();
    if (m.mb_type == H264R_I_PCM) {
        lv.resize(128 + mwc * mhc);
        uint8_t* raw = reinterpret_cast<uint8_t*>(lv.data());
        for (int y = 0; y < 16; ++y)
            for (int x = 0; x < 16; ++x) raw[y * 16 + x] = (uint8_t)cof[0][y][x];
        for (int p = 0; p < 2; ++p)
            for (int y = 0; y < mhc; ++y)
                for (int x = 0; x < mwc; ++x) raw[256 + p * mwc * mhc + y * mwc + x] = (uint8_t)cof[1 + p][y][x];
    } else if (cf == 3 || cf == 0) {
        // three luma-like blocks (include/h264r.h, 4:4:4): Y, Cb, Cr; 4:0:0 the luma one
        for (int p = 0; p < (cf == 3 ? 3 : 1); ++p) {
            for (int b8 = 0; b8 < 4; ++b8) {
                if (!((cbpl >> b8) & 1)) continue;
                const int x8 = (b8 & 1) * 8, y8 = (b8 >> 1) * 8;
                if (!m.t8) {
                    for (int k = 0; k < 4; ++k)
                        for (int i = 0; i < 16; ++i)
                            lv.push_back((int16_t)cof[p][y8 + (k >> 1) * 4 + i / 4][x8 + (k & 1) * 4 + i % 4]);
                    if (m.mb_type == H264R_I_16x16)
                        for (int k = 0; k < 4; ++k) lv[lv.size() - 64 + k * 16] = 0;
                } else {
                    for (int i = 0; i < 64; ++i) lv.push_back((int16_t)cof[p][y8 + i / 8][x8 + i % 8]);
                }
            }
            if (m.mb_type == H264R_I_16x16)
                for (int i = 0; i < 16; ++i) lv.push_back((int16_t)cof[p][(i / 4) * 4][(i % 4) * 4]);
        }
    } else if (cf == 2) {
        // the 4:2:2 level block (include/h264r.h): the luma part, then chroma AC, then DC
        for (int b8 = 0; b8 < 4; ++b8) {
            if (!((cbpl >> b8) & 1)) continue;
            const int x8 = (b8 & 1) * 8, y8 = (b8 >> 1) * 8;
            if (!m.t8) {
                for (int k = 0; k < 4; ++k)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back((int16_t)cof[0][y8 + (k >> 1) * 4 + i / 4][x8 + (k & 1) * 4 + i % 4]);
                if (m.mb_type == H264R_I_16x16)
                    for (int k = 0; k < 4; ++k) lv[lv.size() - 64 + k * 16] = 0;
            } else {
                for (int i = 0; i < 64; ++i) lv.push_back((int16_t)cof[0][y8 + i / 8][x8 + i % 8]);
            }
        }
        if (m.mb_type == H264R_I_16x16)
            for (int i = 0; i < 16; ++i) lv.push_back((int16_t)cof[0][(i / 4) * 4][(i % 4) * 4]);
        if (cbpc == 2)
            for (int p = 1; p <= 2; ++p)
                for (int bb = 0; bb < 8; ++bb)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back(i == 0 ? 0 : (int16_t)cof[p][(bb >> 1) * 4 + i / 4][(bb & 1) * 4 + i % 4]);
        if (cbpc)
            for (int p = 1; p <= 2; ++p)
                for (int q = 0; q < 8; ++q) lv.push_back((int16_t)cof[p][(q / 2) * 4][(q % 2) * 4]);
    } else {
        for (int b8 = 0; b8 < 4; ++b8) {
            if (!((cbpl >> b8) & 1)) continue;
            const int x8 = (b8 & 1) * 8, y8 = (b8 >> 1) * 8;
            if (!m.t8) {
                for (int k = 0; k < 4; ++k)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back((int16_t)cof[0][y8 + (k >> 1) * 4 + i / 4][x8 + (k & 1) * 4 + i % 4]);
                if (m.mb_type == H264R_I_16x16)
                    for (int k = 0; k < 4; ++k) lv[lv.size() - 64 + k * 16] = 0;
            } else {
                for (int i = 0; i < 64; ++i) lv.push_back((int16_t)cof[0][y8 + i / 8][x8 + i % 8]);
            }
        }
        if (cbpc == 2)
            for (int p = 1; p <= 2; ++p)
                for (int bb = 0; bb < 4; ++bb)
                    for (int i = 0; i < 16; ++i)
                        lv.push_back(i == 0 ? 0 : (int16_t)cof[p][(bb >> 1) * 4 + i / 4][(bb & 1) * 4 + i % 4]);
        if (m.mb_type == H264R_I_16x16)
            for (int i = 0; i < 16; ++i) lv.push_back((int16_t)cof[0][(i / 4) * 4][(i % 4) * 4]);
        if (cbpc)
            for (int p = 1; p <= 2; ++p)
                for (int q = 0; q < 4; ++q) lv.push_back((int16_t)cof[p][(q / 2) * 4][(q % 2) * 4]);
    }
    const Motion& M = *D.mot_;
    for (int k = 0; k < 16; ++k) {
        const size_t e = M.at(mbx * 4 + k % 4, mby * 4 + k / 4);
        for (int l = 0; l < 2; ++l) {
            st.mv[l][k] = (uint32_t)(uint16_t)M.mvx[l][e] | (uint32_t)(uint16_t)M.mvy[l][e] << 16;
            st.ref[l][k] = M.ref_pic[l][e] >= 0 ? M.ref_idx[l][e] : (int8_t)-1;
        }
    }
    D.seen_[si] = 1;
}

}  // namespace
}  // namespace h264p

struct h264p_dec {
    h264p::Decoder d;
    explicit h264p_dec(int device) : d(device) {}
};

extern "C" {

int h264p_create(h264p_dec** out, int device)
{
    if (!out) return H264R_EINVAL;
    *out = nullptr;
    try {
        *out = new h264p_dec(device);
    } catch (...) {
        return H264R_ENOMEM;
    }
    return H264R_OK;
}

int h264p_destroy(h264p_dec* dec)
{
    delete dec;
    return H264R_OK;
}

int h264p_decode(h264p_dec* dec, const uint8_t* data, size_t size, h264p_output_fn out, void* user)
{
    if (!dec || (!data && size)) return H264R_EINVAL;
    try {
        return dec->d.decode(data, size, out, user);
    } catch (const std::bad_alloc&) {
        return H264R_ENOMEM;
    }
}

const char* h264p_last_error(const h264p_dec* dec) { return dec ? dec->d.err.c_str() : "no decoder"; }

}  // extern "C"
