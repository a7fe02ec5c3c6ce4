/*
 * probe_cavlc.cc -- TEST INFRASTRUCTURE ONLY (this container; /root/reference).
 *
 * Derives the CAVLC code tables the repo's bitstream writer (tests/h264_writer.py)
 * needs by running the reference decoder's own VLC readers as a black box: every
 * 16-bit pattern is fed to Parser::SyntaxElement::coeff_token / total_zeros /
 * run_before (interpret_se.cc:606-674) and the decoded value + the number of bits the
 * reader consumed are recorded.  The output (JSON on stdout) maps each decoded value
 * to its (length, code) -- H.264 Tables 9-5, 9-7..9-9, 9-10 as the reference reads
 * them.  No reference code or table is copied: the values come from calls.
 *
 * The nested SyntaxElement class is protected inside Parser; this translation unit
 * only widens access (-Dprotected=public on the command line), the layout is unchanged.
 */
#include "global.h"
#include "slice.h"
#include "macroblock.h"

#include <cstdio>
#include <map>
#include <utility>

using namespace vio::h264;

int main()
{
    sps_t* sps = new sps_t();
    pps_t* pps = new pps_t();
    sps->ChromaArrayType = 1;
    slice_t* sl = new slice_t();
    sl->active_sps = sps; sl->active_pps = pps;
    sl->parser.dp_mode = 0;
    mb_t* mb = new mb_t();
    mb->p_Slice = sl;
    mb->is_intra_block = 1;
    InterpreterRbsp& dp = sl->parser.partArr[0];
    Parser::SyntaxElement se(*mb);

    auto feed = [&](unsigned pat) {
        dp.rbsp_byte[0] = (uint8_t)(pat >> 8);
        dp.rbsp_byte[1] = (uint8_t)pat;
        dp.rbsp_byte[2] = 0xFF; dp.rbsp_byte[3] = 0xFF;   /* never consumed: codes are <= 16 bits */
        dp.num_bytes_in_rbsp = 4;
        dp.frame_bitoffset = 0;
    };
    printf("{\n");
    /* coeff_token: nC classes 0 (0..1), 2 (2..3), 4 (4..7), -1 (chroma DC 4:2:0), -2 (4:2:2) */
    const int ncs[5] = {0, 2, 4, -1, -2};
    printf("\"coeff_token\": {\n");
    for (int t = 0; t < 5; ++t) {
        std::map<int, std::pair<int, unsigned>> m;
        for (unsigned pat = 0; pat < 65536; ++pat) {
            feed(pat);
            int v = se.coeff_token(ncs[t]);
            int len = dp.frame_bitoffset;
            if (len <= 0 || len > 16) continue;
            unsigned code = pat >> (16 - len);
            if (!m.count(v)) m[v] = {len, code};
        }
        printf("  \"%d\": [", ncs[t]);
        bool first = true;
        for (auto& kv : m) {
            printf("%s[%d, %d, %d, %u]", first ? "" : ", ", kv.first >> 2, kv.first & 3, kv.second.first, kv.second.second);
            first = false;
        }
        printf("]%s\n", t < 4 ? "," : "");
    }
    printf("},\n\"total_zeros\": {\n");
    /* yuv 0: chroma DC 4:2:0 (tzVlcIndex 1..3), 1: chroma DC 4:2:2 (1..7), 2: 4x4 blocks (1..15) */
    const int tzmax[3] = {3, 7, 15};
    for (int yuv = 0; yuv < 3; ++yuv) {
        printf("  \"%d\": {", yuv);
        for (int tz = 1; tz <= tzmax[yuv]; ++tz) {
            std::map<int, std::pair<int, unsigned>> m;
            for (unsigned pat = 0; pat < 65536; ++pat) {
                feed(pat);
                int v = se.total_zeros(yuv, tz);
                int len = dp.frame_bitoffset;
                if (len <= 0 || len > 16) continue;
                if (!m.count(v)) m[v] = {len, pat >> (16 - len)};
            }
            printf("%s\"%d\": [", tz > 1 ? ", " : "", tz);
            bool first = true;
            for (auto& kv : m) {
                printf("%s[%d, %d, %u]", first ? "" : ", ", kv.first, kv.second.first, kv.second.second);
                first = false;
            }
            printf("]");
        }
        printf("}%s\n", yuv < 2 ? "," : "");
    }
    printf("},\n\"run_before\": {");
    for (int zl = 1; zl <= 7; ++zl) {
        std::map<int, std::pair<int, unsigned>> m;
        for (unsigned pat = 0; pat < 65536; ++pat) {
            feed(pat);
            int v = se.run_before((uint8_t)zl);
            int len = dp.frame_bitoffset;
            if (len <= 0 || len > 16) continue;
            if (!m.count(v)) m[v] = {len, pat >> (16 - len)};
        }
        printf("%s\"%d\": [", zl > 1 ? ", " : "", zl);
        bool first = true;
        for (auto& kv : m) {
            printf("%s[%d, %d, %u]", first ? "" : ", ", kv.first, kv.second.first, kv.second.second);
            first = false;
        }
        printf("]");
    }
    printf("},\n\"cbp_me\": {");
    /* coded_block_pattern me(v), chroma_format_idc 1 (interpret_se.cc:389-417): codeNum -> cbp,
       intra then inter; the codeNum is written as ue(v) */
    sps->chroma_format_idc = 1;
    for (int inter = 0; inter < 2; ++inter) {
        mb->is_intra_block = !inter;
        printf("%s\"%s\": [", inter ? ", " : "", inter ? "inter" : "intra");
        for (unsigned k = 0; k < 48; ++k) {
            unsigned v = k + 1; int nb = 0;
            while ((v >> nb) > 1) ++nb;                     /* ue(v): nb zeros, then v in nb + 1 bits */
            unsigned pat = v << (15 - 2 * nb);               /* 2 nb + 1 <= 11 bits, left-aligned in 16 */
            feed(pat);
            printf("%s%d", k ? ", " : "", (int)se.coded_block_pattern());
        }
        printf("]");
    }
    /* the same for ChromaArrayType 0 / 3 (4:4:4: no chroma CBP, codeNum 0..15, the table's other half) */
    sps->chroma_format_idc = 3;
    printf("},\n\"cbp_me_444\": {");
    for (int inter = 0; inter < 2; ++inter) {
        mb->is_intra_block = !inter;
        printf("%s\"%s\": [", inter ? ", " : "", inter ? "inter" : "intra");
        for (unsigned k = 0; k < 16; ++k) {
            unsigned v = k + 1; int nb = 0;
            while ((v >> nb) > 1) ++nb;
            unsigned pat = v << (15 - 2 * nb);
            feed(pat);
            printf("%s%d", k ? ", " : "", (int)se.coded_block_pattern());
        }
        printf("]");
    }
    mb->is_intra_block = 1;
    printf("}\n}\n");
    return 0;
}
