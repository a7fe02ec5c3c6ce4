/*
 * probe_cabac.cc -- TEST INFRASTRUCTURE ONLY (this container; /root/reference).
 *
 * What the repo's CABAC bitstream writer (tests/h264_writer.py) needs from the reference
 * decoder, taken from the compiled reference (tests/golden/make_cabac_tables.py turns the
 * JSON on stdout into tests/golden/cabac_tables.json):
 *
 *  - the context variables after cabac_contexts_t::init(slice_type, cabac_init_idc, QP)
 *    (bitstream_cabac.cc:1215-1264) for I, P and B slices, every cabac_init_idc and every
 *    SliceQpY 0..51, as (pStateIdx, valMPS) per context in the struct's own order
 *    (bitstream_cabac.h:61-83, field offsets printed alongside) -- called, not read;
 *  - the arithmetic engine's state tables, by driving cabac_engine_t::decode_decision
 *    (interpret.cc:318-341) as a black box: for every (pStateIdx, qCodIRangeIdx) one
 *    forced LPS decision gives rangeTabLPS (the new codIRange shifted back by the bits
 *    RenormD read) and transIdxLPS, one forced MPS decision gives transIdxMPS;
 *  - the residual context maps of residual_block_cabac (interpret_residual.cc:175-270:
 *    position -> ctxIdxInc per block type, and the per-type context offsets).  Those are
 *    file-local tables: this probe links its own copy of interpret_residual.cc compiled
 *    with -Dstatic=extern (oracle/Makefile), which only gives them external linkage.
 */
#include "global.h"
#include "slice.h"
#include "interpret.h"
#include "bitstream_cabac.h"

#include <cstddef>
#include <cstdio>
#include <cstring>

namespace vio {
namespace h264 {
extern const uint8_t pos2ctx_map8x8[];
extern const uint8_t pos2ctx_last8x8[];
extern const uint8_t pos2ctx_map8x8i[];
extern const uint8_t pos2ctx_map4x4[];
extern const uint8_t pos2ctx_map2x4c[];
extern const uint8_t pos2ctx_last4x4[];
extern const uint8_t pos2ctx_last2x4c[];
extern const short type2ctx_bcbp[22];
extern const short type2ctx_map[22];
extern const short type2ctx_one[22];
}
}

using namespace vio::h264;

static void arr8(const char* name, const uint8_t* a, int n, bool comma = true)
{
    printf("\"%s\": [", name);
    for (int i = 0; i < n; ++i) printf("%s%d", i ? ", " : "", a[i]);
    printf("]%s\n", comma ? "," : "");
}
static void arr16(const char* name, const short* a, int n)
{
    printf("\"%s\": [", name);
    for (int i = 0; i < n; ++i) printf("%s%d", i ? ", " : "", a[i]);
    printf("],\n");
}

int main()
{
    printf("{\n");
    // ---- context layout (field, first context, count)
#define F(f) {#f, offsetof(cabac_contexts_t, f) / sizeof(cabac_context_t), sizeof(((cabac_contexts_t*)0)->f) / sizeof(cabac_context_t)}
    struct { const char* name; size_t first, count; } fields[] = {
        F(skip_contexts), F(mb_aff_contexts), F(mb_type_contexts), F(b8_type_contexts), F(transform_size_contexts),
        F(cbp_l_contexts), F(cbp_c_contexts), F(delta_qp_contexts), F(ipr_contexts), F(cipr_contexts),
        F(ref_no_contexts), F(mvd_x_contexts), F(mvd_y_contexts), F(bcbp_contexts), F(map_contexts),
        F(last_contexts), F(one_contexts)};
#undef F
    const int nctx = (int)(sizeof(cabac_contexts_t) / sizeof(cabac_context_t));
    printf("\"num_contexts\": %d,\n\"fields\": [", nctx);
    for (size_t i = 0; i < sizeof(fields) / sizeof(fields[0]); ++i)
        printf("%s[\"%s\", %zu, %zu]", i ? ", " : "", fields[i].name, fields[i].first, fields[i].count);
    printf("],\n");

    // ---- initial states: 255 = not initialised for that slice type
    struct { const char* key; int type, idc; } inits[] = {
        {"I", I_slice, 0}, {"P0", P_slice, 0}, {"P1", P_slice, 1}, {"P2", P_slice, 2},
        {"B0", B_slice, 0}, {"B1", B_slice, 1}, {"B2", B_slice, 2}};
    printf("\"init\": {\n");
    for (size_t t = 0; t < sizeof(inits) / sizeof(inits[0]); ++t) {
        printf("  \"%s\": [", inits[t].key);
        for (int qp = 0; qp < 52; ++qp) {
            cabac_contexts_t c;
            memset(&c, 0xFF, sizeof(c));
            c.init((uint8_t)inits[t].type, (uint8_t)inits[t].idc, (uint8_t)qp);
            const cabac_context_t* v = reinterpret_cast<const cabac_context_t*>(&c);
            printf("%s[", qp ? ",\n    " : "");
            for (int k = 0; k < nctx; ++k)
                printf("%s%d", k ? "," : "", v[k].pStateIdx == 0xFF ? 255 : v[k].pStateIdx | (v[k].valMPS << 6));
            printf("]");
        }
        printf("]%s\n", t + 1 < sizeof(inits) / sizeof(inits[0]) ? "," : "");
    }
    printf("},\n");

    // ---- engine tables through decode_decision
    static uint8_t buf[64];
    InterpreterRbsp dp(64);
    uint8_t lps[64][4], tlps[64], tmps[64];
    for (int s = 0; s < 64; ++s) {
        for (int q = 0; q < 4; ++q) {
            memset(buf, 0, sizeof(buf));
            memcpy(dp.rbsp_byte, buf, sizeof(buf));
            dp.num_bytes_in_rbsp = 64;
            dp.frame_bitoffset = 0;
            cabac_engine_t e;
            e.dp = &dp;
            e.codIRange = (uint16_t)(256 + 64 * q);
            e.codIOffset = (uint16_t)(e.codIRange - 1);            // >= codIRange - rLPS: the LPS path
            cabac_context_t ctx{(uint8_t)s, 0};
            const bool bin = e.decode_decision(&ctx);
            const int nbits = dp.frame_bitoffset;                    // bits RenormD read
            lps[s][q] = (uint8_t)(e.codIRange >> nbits);
            if (q == 0) tlps[s] = ctx.pStateIdx;
            if (bin != 1) { fprintf(stderr, "probe: LPS path not taken\n"); return 1; }
        }
        cabac_engine_t e;
        dp.frame_bitoffset = 0;
        e.dp = &dp;
        e.codIRange = 510;
        e.codIOffset = 0;                                            // the MPS path
        cabac_context_t ctx{(uint8_t)s, 0};
        if (e.decode_decision(&ctx) != 0) { fprintf(stderr, "probe: MPS path not taken\n"); return 1; }
        tmps[s] = ctx.pStateIdx;
    }
    printf("\"rangeTabLPS\": [");
    for (int s = 0; s < 64; ++s) printf("%s[%d, %d, %d, %d]", s ? ", " : "", lps[s][0], lps[s][1], lps[s][2], lps[s][3]);
    printf("],\n");
    arr8("transIdxLPS", tlps, 64);
    arr8("transIdxMPS", tmps, 64);

    // ---- residual context maps
    arr8("pos2ctx_map8x8", pos2ctx_map8x8, 64);
    arr8("pos2ctx_map8x8_field", pos2ctx_map8x8i, 64);   // field-coded blocks (pos2ctx_map[1])
    arr8("pos2ctx_last8x8", pos2ctx_last8x8, 64);
    arr8("pos2ctx_map4x4", pos2ctx_map4x4, 16);
    arr8("pos2ctx_map2x4c", pos2ctx_map2x4c, 16);
    arr8("pos2ctx_last4x4", pos2ctx_last4x4, 16);
    arr8("pos2ctx_last2x4c", pos2ctx_last2x4c, 16);
    arr16("type2ctx_bcbp", type2ctx_bcbp, 15);
    arr16("type2ctx_map", type2ctx_map, 15);
    printf("\"type2ctx_one\": [");
    for (int i = 0; i < 15; ++i) printf("%s%d", i ? ", " : "", type2ctx_one[i]);
    printf("]\n}\n");
    return 0;
}
