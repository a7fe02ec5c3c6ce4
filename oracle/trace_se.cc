/*
 * trace_se.cc -- TEST INFRASTRUCTURE ONLY (this container): a syntax-element trace of the
 * reference parser for debugging the repo's bitstream writer (tests/h264_writer.py,
 * tests/h264_cabac.py).  oracle/_ref/ldecod_trace is the reference parser + the shim
 * linked with -Wl,--wrap for the parser's syntax-element readers
 * (Parser::SyntaxElement, interpret_se.cc) and the shim's coefficient push: every value
 * the parser decodes is printed to stderr as it is read ("SE <name> <args> = <value>"),
 * then passed on unchanged.  No reference code is modified or copied.
 */
#include <cstdint>
#include <cstdio>

#define SE(ret, fmt, sym, ...) \
    extern "C" ret __real_##sym(void* self);                                                   \
    extern "C" ret __wrap_##sym(void* self) { ret v = __real_##sym(self); fprintf(stderr, "SE %s = %d\n", fmt, (int)v); return v; }

SE(bool, "mb_skip_flag", _ZN3vio4h2646Parser13SyntaxElement12mb_skip_flagEv)
SE(uint8_t, "mb_type", _ZN3vio4h2646Parser13SyntaxElement7mb_typeEv)
SE(uint8_t, "sub_mb_type", _ZN3vio4h2646Parser13SyntaxElement11sub_mb_typeEv)
SE(bool, "transform_size_8x8_flag", _ZN3vio4h2646Parser13SyntaxElement23transform_size_8x8_flagEv)
SE(int8_t, "intra_pred_mode", _ZN3vio4h2646Parser13SyntaxElement15intra_pred_modeEv)
SE(uint8_t, "intra_chroma_pred_mode", _ZN3vio4h2646Parser13SyntaxElement22intra_chroma_pred_modeEv)
SE(uint8_t, "coded_block_pattern", _ZN3vio4h2646Parser13SyntaxElement19coded_block_patternEv)
SE(int8_t, "mb_qp_delta", _ZN3vio4h2646Parser13SyntaxElement11mb_qp_deltaEv)
SE(uint32_t, "mb_skip_run", _ZN3vio4h2646Parser13SyntaxElement11mb_skip_runEv)

extern "C" uint8_t __real__ZN3vio4h2646Parser13SyntaxElement9ref_idx_lEhhh(void*, uint8_t, uint8_t, uint8_t);
extern "C" uint8_t __wrap__ZN3vio4h2646Parser13SyntaxElement9ref_idx_lEhhh(void* s, uint8_t l, uint8_t x, uint8_t y)
{
    uint8_t v = __real__ZN3vio4h2646Parser13SyntaxElement9ref_idx_lEhhh(s, l, x, y);
    fprintf(stderr, "SE ref_idx %d %d %d = %d\n", l, x, y, v);
    return v;
}
extern "C" int16_t __real__ZN3vio4h2646Parser13SyntaxElement5mvd_lEhhhh(void*, uint8_t, uint8_t, uint8_t, uint8_t);
extern "C" int16_t __wrap__ZN3vio4h2646Parser13SyntaxElement5mvd_lEhhhh(void* s, uint8_t l, uint8_t x, uint8_t y, uint8_t c)
{
    int16_t v = __real__ZN3vio4h2646Parser13SyntaxElement5mvd_lEhhhh(s, l, x, y, c);
    fprintf(stderr, "SE mvd %d %d %d %d = %d\n", l, x, y, c, v);
    return v;
}

#define COEFF(name, sym) \
    extern "C" void __real_##sym(void*, void*, int, int, int, int, int);                          \
    extern "C" void __wrap_##sym(void* d, void* mb, int pl, int x0, int y0, int pos, int lev)     \
    { fprintf(stderr, "SE %s %d %d %d %d = %d\n", name, pl, x0, y0, pos, lev); __real_##sym(d, mb, pl, x0, y0, pos, lev); }
COEFF("coeff_luma_dc", _ZN3vio4h2647Decoder13coeff_luma_dcEPNS0_12macroblock_tE10ColorPlaneiiii)
COEFF("coeff_luma_ac", _ZN3vio4h2647Decoder13coeff_luma_acEPNS0_12macroblock_tE10ColorPlaneiiii)
COEFF("coeff_chroma_dc", _ZN3vio4h2647Decoder15coeff_chroma_dcEPNS0_12macroblock_tE10ColorPlaneiiii)
COEFF("coeff_chroma_ac", _ZN3vio4h2647Decoder15coeff_chroma_acEPNS0_12macroblock_tE10ColorPlaneiiii)

// context selections (CtxIdxInc, neighbour.cc), printed as "CTX <name> <args> = <ctxIdxInc>"
extern "C" int __real__ZN3vio4h2649CtxIdxInc5mvd_lEhhhb(void*, uint8_t, uint8_t, uint8_t, bool);
extern "C" int __wrap__ZN3vio4h2649CtxIdxInc5mvd_lEhhhb(void* s, uint8_t l, uint8_t x, uint8_t y, bool c)
{
    int v = __real__ZN3vio4h2649CtxIdxInc5mvd_lEhhhb(s, l, x, y, c);
    fprintf(stderr, "CTX mvd %d %d %d %d = %d\n", l, x, y, (int)c, v);
    return v;
}
extern "C" int __real__ZN3vio4h2649CtxIdxInc12mb_skip_flagEv(void*);
extern "C" int __wrap__ZN3vio4h2649CtxIdxInc12mb_skip_flagEv(void* s)
{
    int v = __real__ZN3vio4h2649CtxIdxInc12mb_skip_flagEv(s);
    fprintf(stderr, "CTX mb_skip_flag = %d\n", v);
    return v;
}
extern "C" int __real__ZN3vio4h2649CtxIdxInc22mb_field_decoding_flagEv(void*);
extern "C" int __wrap__ZN3vio4h2649CtxIdxInc22mb_field_decoding_flagEv(void* s)
{
    int v = __real__ZN3vio4h2649CtxIdxInc22mb_field_decoding_flagEv(s);
    fprintf(stderr, "CTX mb_field_decoding_flag = %d\n", v);
    return v;
}
extern "C" int __real__ZN3vio4h2649CtxIdxInc9ref_idx_lEhhh(void*, uint8_t, uint8_t, uint8_t);
extern "C" int __wrap__ZN3vio4h2649CtxIdxInc9ref_idx_lEhhh(void* s, uint8_t l, uint8_t x, uint8_t y)
{
    int v = __real__ZN3vio4h2649CtxIdxInc9ref_idx_lEhhh(s, l, x, y);
    fprintf(stderr, "CTX ref_idx %d %d %d = %d\n", l, x, y, v);
    return v;
}
