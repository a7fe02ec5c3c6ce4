/*
 * h264r_oracle.c -- TEST INFRASTRUCTURE ONLY (see h264r_oracle.h).
 *
 * Plain-C restatement of the reference's post-entropy reconstruction path on
 * the canonical formats of include/h264r.h.  Every function names the
 * reference lines it follows (H/ = R/src/codec/h264/).  Two documented
 * restatement choices:
 *   (1) motion compensation walks 4x4 blocks with their own mv_info entry
 *       instead of the partition walk of decoder.cc:217-254; with the per-4x4
 *       motion field filled per partition (interpret_mb.cc ref_idx_l/mvd_l)
 *       both give identical samples (per-sample filter, translation-invariant).
 *   (2) get_block_luma's padded-plane reads (inter_prediction.cc:185-339) are
 *       written as per-coordinate clamping; within the 32/12 pads of
 *       picture.cc:27-37 / pad_buf picture.cc:182-205 the two are identical.
 * Both choices are pinned by tests/golden (outputs of the compiled reference).
 */
#include "h264r_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- helpers */
static inline int clip3(int lo, int hi, int x) { return x < lo ? lo : (x > hi ? hi : x); } /* defines.h:48-52 */
static inline int clip1(int hi, int x) { return clip3(0, hi, x); }                         /* defines.h:54-58 */
static inline int iabs(int x) { return x < 0 ? -x : x; }

/* ------------------------------------------------ quant tables (transform.cc:93-170) */
static const int dequant_coef[6][4][4] = {
    {{10, 13, 10, 13}, {13, 16, 13, 16}, {10, 13, 10, 13}, {13, 16, 13, 16}},
    {{11, 14, 11, 14}, {14, 18, 14, 18}, {11, 14, 11, 14}, {14, 18, 14, 18}},
    {{13, 16, 13, 16}, {16, 20, 16, 20}, {13, 16, 13, 16}, {16, 20, 16, 20}},
    {{14, 18, 14, 18}, {18, 23, 18, 23}, {14, 18, 14, 18}, {18, 23, 18, 23}},
    {{16, 20, 16, 20}, {20, 25, 20, 25}, {16, 20, 16, 20}, {20, 25, 20, 25}},
    {{18, 23, 18, 23}, {23, 29, 23, 29}, {18, 23, 18, 23}, {23, 29, 23, 29}}};

/* 8x8 normative scale: v[qp%6][class] (spec Table 8-16 form of transform.cc:121-170). */
static const int dq8_v[6][6] = {
    {20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
    {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};

static int dq8(int m, int i, int j)
{
    /* class of position (i row, j col) */
    if (i % 4 == 0 && j % 4 == 0) return dq8_v[m][0];
    if (i % 2 == 1 && j % 2 == 1) return dq8_v[m][1];
    if (i % 4 == 2 && j % 4 == 2) return dq8_v[m][2];
    if ((i % 4 == 0 && j % 2 == 1) || (i % 2 == 1 && j % 4 == 0)) return dq8_v[m][3];
    if ((i % 4 == 0 && j % 4 == 2) || (i % 4 == 2 && j % 4 == 0)) return dq8_v[m][4];
    return dq8_v[m][5];
}

void oracle_quant_init_flat(h264r_quant* q)
{
    /* Flat_4x4_16 / Flat_8x8_16 (transform.cc:34-50) x dequant_coef (set_quant :264-301) */
    for (int t = 0; t < 2; ++t)
        for (int pl = 0; pl < 3; ++pl)
            for (int m = 0; m < 6; ++m) {
                for (int k = 0; k < 16; ++k)
                    q->scale4x4[t][pl][m][k] = (int16_t)(dequant_coef[m][k / 4][k % 4] * 16);
                for (int k = 0; k < 64; ++k)
                    q->scale8x8[t][pl][m][k] = (int16_t)(dq8(m, k / 8, k % 8) * 16);
            }
}

/* Explicit scaling matrices qmatrix[0..11] (already resolved, raster order: 4x4 lists
 * Intra Y/Cb/Cr, Inter Y/Cb/Cr; 8x8 lists Intra Y, Inter Y, Intra Cb, Inter Cb, Intra Cr,
 * Inter Cr) x dequant_coef, as Transform::set_quant does (transform.cc:259-302). */
void oracle_quant_init_lists(h264r_quant* q, const int32_t* m4 /*[6][16]*/, const int32_t* m8 /*[6][64]*/)
{
    for (int pl = 0; pl < 3; ++pl)
        for (int m = 0; m < 6; ++m) {
            for (int k = 0; k < 16; ++k) {
                q->scale4x4[0][pl][m][k] = (int16_t)(dequant_coef[m][k / 4][k % 4] * m4[pl * 16 + k]);
                q->scale4x4[1][pl][m][k] = (int16_t)(dequant_coef[m][k / 4][k % 4] * m4[(3 + pl) * 16 + k]);
            }
            for (int k = 0; k < 64; ++k) {
                q->scale8x8[0][pl][m][k] = (int16_t)(dq8(m, k / 8, k % 8) * m8[(2 * pl) * 64 + k]);
                q->scale8x8[1][pl][m][k] = (int16_t)(dq8(m, k / 8, k % 8) * m8[(2 * pl + 1) * 64 + k]);
            }
        }
}

/* --------------------------------------------- level block layout (include/h264r.h) */
typedef struct {
    const int16_t* b8[4];   /* NULL when the 8x8 is not coded */
    const int16_t* cac;     /* chroma AC, 2 x nb x 16 levels, or NULL */
    const int16_t* ldc;     /* I16x16 luma DC, 16 levels, or NULL */
    const int16_t* cdc;     /* chroma DC, 2 x nb levels, or NULL */
    int nb;                 /* chroma 4x4 blocks per plane: 4 (4:2:0), 8 (4:2:2) */
} levels_view;

/* cf: chroma_format_idc 1 or 2 (a 4:4:4 picture reaches this code one plane at a time, as
   4:2:0-shaped pictures, decode_444 below) */
static levels_view view_levels(const h264r_mb* mb, const int16_t* pool, int cf)
{
    levels_view v;
    memset(&v, 0, sizeof(v));
    const int16_t* p = pool + mb->coef_off;
    int cbpl = mb->cbp & 15, cbpc = mb->cbp >> 4;
    for (int k = 0; k < 4; ++k)
        if (cbpl & (1 << k)) { v.b8[k] = p; p += 64; }
    if (cf == 2) {          /* 4:2:2 (include/h264r.h): the luma part first, then chroma AC, DC */
        v.nb = 8;
        if (mb->mb_type == H264R_I_16x16) { v.ldc = p; p += 16; }
        if (cbpc == 2) { v.cac = p; p += 256; }
        if (cbpc != 0) { v.cdc = p; p += 16; }
        return v;
    }
    v.nb = 4;
    if (cbpc == 2) { v.cac = p; p += 128; }
    if (mb->mb_type == H264R_I_16x16) { v.ldc = p; p += 16; }
    if (cbpc != 0) { v.cdc = p; p += 8; }
    return v;
}

/* ----------------------------------------------------- transforms (transform.cc) */
static void ihadamard_2x2(int c[2][2], int f[2][2])            /* transform.cc:460-481 */
{
    int e[2][2];
    for (int i = 0; i < 2; ++i) { e[i][0] = c[i][0] + c[i][1]; e[i][1] = c[i][0] - c[i][1]; }
    for (int j = 0; j < 2; ++j) { f[0][j] = e[0][j] + e[1][j]; f[1][j] = e[0][j] - e[1][j]; }
}

static void ihadamard_4x4(int c[4][4], int f[4][4])            /* transform.cc:515-554 */
{
    int e[4][4];
    for (int i = 0; i < 4; ++i) {
        int d0 = c[i][0] + c[i][2], d1 = c[i][0] - c[i][2];
        int d2 = c[i][1] - c[i][3], d3 = c[i][1] + c[i][3];
        e[i][0] = d0 + d3; e[i][1] = d1 + d2; e[i][2] = d1 - d2; e[i][3] = d0 - d3;
    }
    for (int j = 0; j < 4; ++j) {
        int h0 = e[0][j] + e[2][j], h1 = e[0][j] - e[2][j];
        int h2 = e[1][j] - e[3][j], h3 = e[1][j] + e[3][j];
        f[0][j] = h0 + h3; f[1][j] = h1 + h2; f[2][j] = h1 - h2; f[3][j] = h0 - h3;
    }
}

static void inverse_4x4(int d[16][16], int r[16][16], int py, int px)   /* transform.cc:597-641 */
{
    int f[4][4];
    for (int i = 0; i < 4; ++i) {
        int d0 = d[py + i][px + 0], d1 = d[py + i][px + 1];
        int d2 = d[py + i][px + 2], d3 = d[py + i][px + 3];
        int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
        f[i][0] = e0 + e3; f[i][1] = e1 + e2; f[i][2] = e1 - e2; f[i][3] = e0 - e3;
    }
    for (int j = 0; j < 4; ++j) {
        int g0 = f[0][j] + f[2][j], g1 = f[0][j] - f[2][j];
        int g2 = (f[1][j] >> 1) - f[3][j], g3 = f[1][j] + (f[3][j] >> 1);
        r[py + 0][px + j] = (g0 + g3 + 32) >> 6;
        r[py + 1][px + j] = (g1 + g2 + 32) >> 6;
        r[py + 2][px + j] = (g1 - g2 + 32) >> 6;
        r[py + 3][px + j] = (g0 - g3 + 32) >> 6;
    }
}

static void idct8_1d(const int in[8], int out[8])                 /* transform.cc:658-683 */
{
    int e0 = in[0] + in[4];
    int e1 = -in[3] + in[5] - in[7] - (in[7] >> 1);
    int e2 = in[0] - in[4];
    int e3 = in[1] + in[7] - in[3] - (in[3] >> 1);
    int e4 = (in[2] >> 1) - in[6];
    int e5 = -in[1] + in[7] + in[5] + (in[5] >> 1);
    int e6 = in[2] + (in[6] >> 1);
    int e7 = in[3] + in[5] + in[1] + (in[1] >> 1);
    int f0 = e0 + e6, f1 = e1 + (e7 >> 2), f2 = e2 + e4, f3 = e3 + (e5 >> 2);
    int f4 = e2 - e4, f5 = (e3 >> 2) - e5, f6 = e0 - e6, f7 = e7 - (e1 >> 2);
    out[0] = f0 + f7; out[1] = f2 + f5; out[2] = f4 + f3; out[3] = f6 + f1;
    out[4] = f6 - f1; out[5] = f4 - f3; out[6] = f2 - f5; out[7] = f0 - f7;
}

static void inverse_8x8(int d[16][16], int r[16][16], int py, int px)   /* transform.cc:643-733 */
{
    int g[8][8], in[8], out[8];
    for (int i = 0; i < 8; ++i) {
        for (int k = 0; k < 8; ++k) in[k] = d[py + i][px + k];
        idct8_1d(in, g[i]);
    }
    for (int j = 0; j < 8; ++j) {
        for (int k = 0; k < 8; ++k) in[k] = g[k][j];
        idct8_1d(in, out);
        for (int k = 0; k < 8; ++k) r[py + k][px + j] = (out[k] + 32) >> 6;
    }
}

/* Lossless residual DPCM (transform.cc:736-822): a vertical mode accumulates down the
 * columns, a horizontal mode along the rows, any other mode copies.  `vert` / `horz` are
 * the mode values of the block size (0 / 1 for 4x4, 8x8, 16x16; 2 / 1 for chroma). */
static void bypass_block(int r[16][16], int f[16][16], int x0, int y0, int w, int h, int mode, int vert, int horz)
{
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int v = r[y0 + y][x0 + x];
            if (mode == vert && y > 0) v += f[y0 + y - 1][x0 + x];
            else if (mode == horz && x > 0) v += f[y0 + y][x0 + x - 1];
            f[y0 + y][x0 + x] = v;
        }
}

/* TransformBypassModeFlag MBs: levels stay raw (coeff_luma_ac / coeff_chroma_ac skip
 * inverse_quantize, transform.cc:439-441,453-455; transform_luma_dc / transform_chroma_dc
 * do nothing, :827,860), DC levels at the (0,0) of their 4x4 blocks. */
static void load_cof_bypass(const h264r_mb* mb, const int16_t* pool, int cf, int cof[3][16][16])
{
    levels_view v = view_levels(mb, pool, cf);
    int t8 = (mb->flags & H264R_MBF_T8x8) != 0;
    if (v.ldc)
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) cof[0][i * 4][j * 4] = v.ldc[i * 4 + j];
    for (int b8 = 0; b8 < 4; ++b8) {
        const int16_t* blk = v.b8[b8];
        if (!blk) continue;
        for (int b4 = 0; b4 < 4; ++b4)
            for (int pos = 0; pos < 16; ++pos) {
                if (v.ldc && pos == 0 && !t8) continue;
                if (t8) {
                    int k = b4 * 16 + pos;
                    cof[0][(b8 >> 1) * 8 + k / 8][(b8 & 1) * 8 + k % 8] = blk[k];
                } else {
                    int bx = (b8 & 1) * 2 + (b4 & 1), by = (b8 >> 1) * 2 + (b4 >> 1);
                    cof[0][by * 4 + pos / 4][bx * 4 + pos % 4] = blk[b4 * 16 + pos];
                }
            }
    }
    for (int pl = 1; pl <= 2; ++pl) {
        if (v.cdc)
            for (int i = 0; i < v.nb / 2; ++i)
                for (int j = 0; j < 2; ++j) cof[pl][i * 4][j * 4] = v.cdc[(pl - 1) * v.nb + i * 2 + j];
        if (v.cac)
            for (int b = 0; b < v.nb; ++b)
                for (int pos = 1; pos < 16; ++pos)
                    cof[pl][(b / 2) * 4 + pos / 4][(b % 2) * 4 + pos % 4] = v.cac[(pl - 1) * v.nb * 16 + b * 16 + pos];
    }
}

/* Coefficient push: coeff_luma_ac/coeff_chroma_ac + inverse_quantize (transform.cc:394-456),
 * transform_luma_dc (:825-856), transform_chroma_dc (:858-910). */
static void load_cof(const h264r_mb* mb, const int16_t* pool, const h264r_quant* q, int cf, int cof[3][16][16])
{
    memset(cof, 0, sizeof(int) * 3 * 16 * 16);
    if (mb->flags & H264R_MBF_BYPASS) { load_cof_bypass(mb, pool, cf, cof); return; }
    levels_view v = view_levels(mb, pool, cf);
    int inter = (mb->flags & H264R_MBF_INTRA) ? 0 : 1;
    int t8 = (mb->flags & H264R_MBF_T8x8) != 0;
    int i16 = mb->mb_type == H264R_I_16x16;

    if (i16) {
        int c[4][4], f[4][4];
        int qP = mb->qp_scaled[0];
        int scale = q->scale4x4[0][0][qP % 6][0];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) c[i][j] = v.ldc[i * 4 + j];
        ihadamard_4x4(c, f);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                if (qP >= 36)
                    cof[0][i * 4][j * 4] = (f[i][j] * scale) * (1 << (qP / 6 - 6));
                else
                    cof[0][i * 4][j * 4] = (f[i][j] * scale + (1 << (5 - qP / 6))) >> (6 - qP / 6);
            }
    }
    {
        int qp = mb->qp_scaled[0], per = qp / 6, rem = qp % 6;
        for (int b8 = 0; b8 < 4; ++b8) {
            const int16_t* blk = v.b8[b8];
            if (!blk) continue;
            if (!t8) {
                for (int b4 = 0; b4 < 4; ++b4) {
                    int bx = (b8 & 1) * 2 + (b4 & 1), by = (b8 >> 1) * 2 + (b4 >> 1);
                    for (int pos = i16 ? 1 : 0; pos < 16; ++pos) {
                        int lev = blk[b4 * 16 + pos];
                        if (!lev) continue;
                        int s = q->scale4x4[inter][0][rem][pos];
                        cof[0][by * 4 + pos / 4][bx * 4 + pos % 4] = ((lev * s) * (1 << per) + 8) >> 4;
                    }
                }
            } else {
                int x0 = (b8 & 1) * 8, y0 = (b8 >> 1) * 8;
                for (int pos = 0; pos < 64; ++pos) {
                    int lev = blk[pos];
                    if (!lev) continue;
                    int s = q->scale8x8[inter][0][rem][pos];
                    cof[0][y0 + pos / 8][x0 + pos % 8] = ((lev * s) * (1 << per) + 32) >> 6;
                }
            }
        }
    }
    for (int pl = 1; pl <= 2; ++pl) {
        int qP = mb->qp_scaled[pl];
        if (v.cdc && v.nb == 4) {
            int c[2][2], f[2][2];
            int scale = q->scale4x4[inter][pl][qP % 6][0];
            for (int k = 0; k < 4; ++k) c[k / 2][k % 2] = v.cdc[(pl - 1) * 4 + k];
            ihadamard_2x2(c, f);
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j)
                    cof[pl][i * 4][j * 4] = ((f[i][j] * scale) * (1 << (qP / 6))) >> 5;
        } else if (v.cdc) {
            /* 4:2:2: ihadamard_2x4 (transform.cc:483-513) and the dequantisation of :890-907 -- with
               qP = qp_scaled[pl] as the reference has it, where 8.5.11.2 uses QP'c + 3 (the
               reference's doc/bugs-jm-18.5.txt item 11 drops JM's + 3 on purpose) */
            int c[4][2], e[4][2], f[4][2];
            int scale = q->scale4x4[inter][pl][qP % 6][0];
            for (int k = 0; k < 8; ++k) c[k / 2][k % 2] = v.cdc[(pl - 1) * 8 + k];
            for (int i = 0; i < 4; ++i) { e[i][0] = c[i][0] + c[i][1]; e[i][1] = c[i][0] - c[i][1]; }
            for (int j = 0; j < 2; ++j) {
                int h0 = e[0][j] + e[2][j], h1 = e[0][j] - e[2][j], h2 = e[1][j] - e[3][j], h3 = e[1][j] + e[3][j];
                f[0][j] = h0 + h3; f[1][j] = h1 + h2; f[2][j] = h1 - h2; f[3][j] = h0 - h3;
            }
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 2; ++j)
                    cof[pl][i * 4][j * 4] = qP >= 36 ? (f[i][j] * scale) * (1 << (qP / 6 - 6))
                                                     : (f[i][j] * scale + (1 << (5 - qP / 6))) >> (6 - qP / 6);
        }
        if (v.cac) {
            const int16_t* blk = v.cac + (pl - 1) * v.nb * 16;
            for (int b = 0; b < v.nb; ++b)
                for (int pos = 1; pos < 16; ++pos) {
                    int lev = blk[b * 16 + pos];
                    if (!lev) continue;
                    int s = q->scale4x4[inter][pl][qP % 6][pos];
                    cof[pl][(b / 2) * 4 + pos / 4][(b % 2) * 4 + pos % 4] =
                        ((lev * s) * (1 << (qP / 6)) + 8) >> 4;
                }
        }
    }
}


/* --------------------------------------------------------------- picture state */
typedef struct {
    const oracle_picture* p;
    int wmb, hmb, W, H, Wc, Hc, W4, H4;
    int cf, MHc;           /* chroma_format_idc (1, 2) and MbHeightC (8, 16) */
    int fld, bot;          /* a field picture (shr.field_pic_flag) and its parity (bottom_field_flag) */
    int mbaff;             /* an MBAFF frame (shr.MbaffFrameFlag): MB pairs, records in storage rows */
    int16_t* slice_nr;     /* slice_nr per MB, -1 until decoded (reset_mbs slice_data.cc:55, mb.init :465) */
    uint8_t  (*strength_ver)[4][16];   /* mb_t::strength_ver, deblock.cc:80 */
    uint8_t  (*strength_hor)[4][16];   /* mb_t::strength_hor, deblock.cc:159 */
    uint8_t  (*fver)[2][4];            /* filterVerEdgeFlag[chroma][edge], deblock.cc:255-278 */
    uint8_t  (*fhor)[2][4];            /* filterHorEdgeFlag */
    uint8_t  (*strength_hor4)[16];     /* MBAFF: strength_hor[4], the second field edge (deblock.cc:285-286) */
    uint8_t  (*fhor4)[2];              /* MBAFF: filterHorEdgeFlag[chroma][4] (:262-263) */
} pstate;

static inline const h264r_mb* mb_at(const pstate* s, int addr) { return &s->p->mbs[addr]; }
static inline const h264r_slice* slice_of(const pstate* s, const h264r_mb* mb) { return &s->p->slices[mb->slice]; }

/* Neighbour::get_neighbour for non-MBAFF frames (neighbour.cc:123-173) followed by the
 * callers' slice check (e.g. intra_prediction.cc:145-152).  Returns the MB address or -1;
 * (*ax,*ay) receive the absolute sample location. */
static inline int is_field_mb(const pstate* s, int addr) { return (s->p->mbs[addr].flags & H264R_MBF_FIELD) != 0; }

/* MBAFF frames.  `addr` is the storage index (mb_t::mb: row 2 pair_row + bottom, include/h264r.h);
 * the planes hold the frame as it is after MbAffPostProc (deblock.cc:581-620), so a field MB's
 * row y is frame row 2 y (+ 1 for the bottom MB) of its pair.  Neighbour::get_location (neighbour.cc:
 * 47-77) of sample (ox, oy) of MB addr, in frame coordinates: */
static void mbaff_loc(const pstate* s, int addr, int maxW, int maxH, int ox, int oy, int* x, int* y)
{
    const int mby = addr / s->wmb, b = mby & 1;
    *x = (addr % s->wmb) * maxW + ox;
    *y = (mby >> 1) * 2 * maxH + (is_field_mb(s, addr) ? b + 2 * oy : b * maxH + oy);
}
/* Neighbour::get_mb / get_neighbour (neighbour.cc:175-227): the MB holding frame sample (x, y) --
 * the bottom MB of its pair when the pair is a field pair and y is odd, or a frame pair and y is in
 * its lower half -- or -1 outside the picture; *ly = the sample's row inside that MB */
static int mbaff_mb_at(const pstate* s, int maxW, int maxH, int x, int y, int* ly)
{
    if (x < 0 || x >= s->wmb * maxW || y < 0 || y >= s->hmb * maxH) return -1;
    const int top = ((y / (2 * maxH)) * 2) * s->wmb + x / maxW, r = y % (2 * maxH);
    const int f = is_field_mb(s, top);
    const int b = f ? (y & 1) : r >= maxH;
    if (ly) *ly = f ? r / 2 : r % maxH;
    return top + b * s->wmb;
}

static int get_neighbour(const pstate* s, int chroma, int addr, int ox, int oy, int* ax, int* ay)
{
    int maxW = chroma ? 8 : 16, maxH = chroma ? s->MHc : 16;
    if (s->mbaff) {
        int x, y;
        mbaff_loc(s, addr, maxW, maxH, ox, oy, &x, &y);
        int n = mbaff_mb_at(s, maxW, maxH, x, y, NULL);
        if (n < 0 || s->slice_nr[n] != s->slice_nr[addr]) return -1;
        *ax = x; *ay = y;
        return n;
    }
    int x = (addr % s->wmb) * maxW + ox, y = (addr / s->wmb) * maxH + oy;
    if (x < 0 || x >= s->wmb * maxW || y < 0 || y >= s->hmb * maxH) return -1;
    int n = (y / maxH) * s->wmb + (x / maxW);
    if (s->slice_nr[n] != s->slice_nr[addr]) return -1;
    *ax = x; *ay = y;
    return n;
}

static inline int is_intra(const pstate* s, int addr) { return (mb_at(s, addr)->flags & H264R_MBF_INTRA) != 0; }

/* --------------------------------------------------------- intra prediction */
typedef struct { int avail[4]; int smp[18 * 18]; int stride; } nbr_t;   /* samples p(x,y), x,y >= -1 */
#define P(n, x, y) ((n)->smp[((y) + 1) * (n)->stride + ((x) + 1)])

/* Intra4x4 ctor (intra_prediction.cc:137-187) and Intra8x8 ctor (:359-411), size 4 or 8. */
static void gather_nxn(const pstate* s, int addr, int size, int xO, int yO, const uint8_t* img, int pitch, nbr_t* n)
{
    int cip = s->p->pic->constrained_intra_pred;
    int bx = 0, by = 0, cx = 0, cy = 0, dx = 0, dy = 0;
    int nA[8], ax[8] = {0}, ay[8] = {0};          /* each row's own sample (an MBAFF pair's rows) */
    for (int i = 0; i < size; ++i) nA[i] = get_neighbour(s, 0, addr, xO - 1, yO + i, &ax[i], &ay[i]);
    int nB = get_neighbour(s, 0, addr, xO, yO - 1, &bx, &by);
    int nC = get_neighbour(s, 0, addr, xO + size, yO - 1, &cx, &cy);
    int nD = get_neighbour(s, 0, addr, xO - 1, yO - 1, &dx, &dy);
    if (size == 4 && xO == 4 && (yO == 4 || yO == 12)) nC = -1;   /* :154 */
    if (size == 8 && xO == 8 && yO == 8) nC = -1;                  /* :376 */
    n->stride = 18;
    if (cip) {
        n->avail[0] = 1;
        for (int i = 0; i < size; ++i) n->avail[0] &= nA[i] >= 0 && is_intra(s, nA[i]);
        n->avail[1] = nB >= 0 && is_intra(s, nB);
        n->avail[2] = nC >= 0 && is_intra(s, nC);
        n->avail[3] = nD >= 0 && is_intra(s, nD);
    } else {
        n->avail[0] = nA[0] >= 0; n->avail[1] = nB >= 0;
        n->avail[2] = nC >= 0;    n->avail[3] = nD >= 0;
    }
    if (n->avail[3]) P(n, -1, -1) = img[dy * pitch + dx];
    if (n->avail[0])
        for (int y = 0; y < size; ++y) P(n, -1, y) = img[ay[y] * pitch + ax[y]];
    if (n->avail[1]) {
        for (int x = 0; x < size; ++x) P(n, x, -1) = img[by * pitch + bx + x];
        for (int x = size; x < 2 * size; ++x)
            P(n, x, -1) = n->avail[2] ? img[cy * pitch + cx + (x - size)] : P(n, size - 1, -1);
        n->avail[2] = n->avail[1];
    }
}

static void pred_4x4(nbr_t* n, int mode, int pred[16][16], int xO, int yO)   /* :189-346 */
{
#define PR(x, y) pred[yO + (y)][xO + (x)]
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            int v;
            switch (mode) {
            case 0: v = P(n, x, -1); break;
            case 1: v = P(n, -1, y); break;
            case 2: {
                int aA = n->avail[0], aB = n->avail[1], sum = 0;
                if (aA || aB) {
                    if (aA) for (int k = 0; k < 4; ++k) sum += P(n, -1, k);
                    if (aB) for (int k = 0; k < 4; ++k) sum += P(n, k, -1);
                    v = (sum + (aA ? 2 : 0) + (aB ? 2 : 0)) >> (1 + aA + aB);
                } else v = 128;
                break; }
            case 3:
                if (x == 3 && y == 3) v = (P(n, 6, -1) + 3 * P(n, 7, -1) + 2) >> 2;
                else v = (P(n, x + y, -1) + 2 * P(n, x + y + 1, -1) + P(n, x + y + 2, -1) + 2) >> 2;
                break;
            case 4:
                if (x > y) v = (P(n, x - y - 2, -1) + 2 * P(n, x - y - 1, -1) + P(n, x - y, -1) + 2) >> 2;
                else if (x < y) v = (P(n, -1, y - x - 2) + 2 * P(n, -1, y - x - 1) + P(n, -1, y - x) + 2) >> 2;
                else v = (P(n, 0, -1) + 2 * P(n, -1, -1) + P(n, -1, 0) + 2) >> 2;
                break;
            case 5: {
                int z = 2 * x - y;
                if (z >= 0 && (z & 1) == 0) v = (P(n, x - (y >> 1) - 1, -1) + P(n, x - (y >> 1), -1) + 1) >> 1;
                else if (z >= 0) v = (P(n, x - (y >> 1) - 2, -1) + 2 * P(n, x - (y >> 1) - 1, -1) + P(n, x - (y >> 1), -1) + 2) >> 2;
                else if (z == -1) v = (P(n, -1, 0) + 2 * P(n, -1, -1) + P(n, 0, -1) + 2) >> 2;
                else v = (P(n, -1, y - 2 * x - 1) + 2 * P(n, -1, y - 2 * x - 2) + P(n, -1, y - 2 * x - 3) + 2) >> 2;
                break; }
            case 6: {
                int z = 2 * y - x;
                if (z >= 0 && (z & 1) == 0) v = (P(n, -1, y - (x >> 1) - 1) + P(n, -1, y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (P(n, -1, y - (x >> 1) - 2) + 2 * P(n, -1, y - (x >> 1) - 1) + P(n, -1, y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (P(n, -1, 0) + 2 * P(n, -1, -1) + P(n, 0, -1) + 2) >> 2;
                else v = (P(n, x - 2 * y - 1, -1) + 2 * P(n, x - 2 * y - 2, -1) + P(n, x - 2 * y - 3, -1) + 2) >> 2;
                break; }
            case 7:
                if ((y & 1) == 0) v = (P(n, x + (y >> 1), -1) + P(n, x + (y >> 1) + 1, -1) + 1) >> 1;
                else v = (P(n, x + (y >> 1), -1) + 2 * P(n, x + (y >> 1) + 1, -1) + P(n, x + (y >> 1) + 2, -1) + 2) >> 2;
                break;
            default: {   /* 8: horizontal up */
                int z = x + 2 * y;
                if (z < 5 && (z & 1) == 0) v = (P(n, -1, y + (x >> 1)) + P(n, -1, y + (x >> 1) + 1) + 1) >> 1;
                else if (z < 5) v = (P(n, -1, y + (x >> 1)) + 2 * P(n, -1, y + (x >> 1) + 1) + P(n, -1, y + (x >> 1) + 2) + 2) >> 2;
                else if (z == 5) v = (P(n, -1, 2) + 3 * P(n, -1, 3) + 2) >> 2;
                else v = P(n, -1, 3);
                break; }
            }
            PR(x, y) = v;
        }
#undef PR
}

/* Intra8x8::filtering (intra_prediction.cc:413-447): n holds po(), returns p() in f. */
static void filter_8x8(const nbr_t* n, nbr_t* f)
{
    int aA = n->avail[0], aB = n->avail[1], aD = n->avail[3];
    *f = *n;
    if (aB) {
        P(f, 0, -1) = aD ? (P(n, -1, -1) + 2 * P(n, 0, -1) + P(n, 1, -1) + 2) >> 2
                         : (3 * P(n, 0, -1) + P(n, 1, -1) + 2) >> 2;
        for (int x = 1; x < 15; ++x) P(f, x, -1) = (P(n, x - 1, -1) + 2 * P(n, x, -1) + P(n, x + 1, -1) + 2) >> 2;
        P(f, 15, -1) = (P(n, 14, -1) + 3 * P(n, 15, -1) + 2) >> 2;
    }
    if (aD) {
        if (aA && aB) P(f, -1, -1) = (P(n, 0, -1) + 2 * P(n, -1, -1) + P(n, -1, 0) + 2) >> 2;
        else if (aB) P(f, -1, -1) = (3 * P(n, -1, -1) + P(n, 0, -1) + 2) >> 2;
        else if (aA) P(f, -1, -1) = (3 * P(n, -1, -1) + P(n, -1, 0) + 2) >> 2;
        else P(f, -1, -1) = P(n, -1, -1);
    }
    if (aA) {
        P(f, -1, 0) = aD ? (P(n, -1, -1) + 2 * P(n, -1, 0) + P(n, -1, 1) + 2) >> 2
                         : (3 * P(n, -1, 0) + P(n, -1, 1) + 2) >> 2;
        for (int y = 1; y < 7; ++y) P(f, -1, y) = (P(n, -1, y - 1) + 2 * P(n, -1, y) + P(n, -1, y + 1) + 2) >> 2;
        P(f, -1, 7) = (P(n, -1, 6) + 3 * P(n, -1, 7) + 2) >> 2;
    }
}

static void pred_8x8(nbr_t* n, int mode, int pred[16][16], int xO, int yO)   /* :449-606 */
{
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
            int v;
            switch (mode) {
            case 0: v = P(n, x, -1); break;
            case 1: v = P(n, -1, y); break;
            case 2: {
                int aA = n->avail[0], aB = n->avail[1], sum = 0;
                if (aA || aB) {
                    if (aA) for (int k = 0; k < 8; ++k) sum += P(n, -1, k);
                    if (aB) for (int k = 0; k < 8; ++k) sum += P(n, k, -1);
                    v = (sum + (aA ? 4 : 0) + (aB ? 4 : 0)) >> (2 + aA + aB);
                } else v = 128;
                break; }
            case 3:
                if (x == 7 && y == 7) v = (P(n, 14, -1) + 3 * P(n, 15, -1) + 2) >> 2;
                else v = (P(n, x + y, -1) + 2 * P(n, x + y + 1, -1) + P(n, x + y + 2, -1) + 2) >> 2;
                break;
            case 4:
                if (x > y) v = (P(n, x - y - 2, -1) + 2 * P(n, x - y - 1, -1) + P(n, x - y, -1) + 2) >> 2;
                else if (x < y) v = (P(n, -1, y - x - 2) + 2 * P(n, -1, y - x - 1) + P(n, -1, y - x) + 2) >> 2;
                else v = (P(n, 0, -1) + 2 * P(n, -1, -1) + P(n, -1, 0) + 2) >> 2;
                break;
            case 5: {
                int z = 2 * x - y;
                if (z >= 0 && (z & 1) == 0) v = (P(n, x - (y >> 1) - 1, -1) + P(n, x - (y >> 1), -1) + 1) >> 1;
                else if (z >= 0) v = (P(n, x - (y >> 1) - 2, -1) + 2 * P(n, x - (y >> 1) - 1, -1) + P(n, x - (y >> 1), -1) + 2) >> 2;
                else if (z == -1) v = (P(n, -1, 0) + 2 * P(n, -1, -1) + P(n, 0, -1) + 2) >> 2;
                else v = (P(n, -1, y - 2 * x - 1) + 2 * P(n, -1, y - 2 * x - 2) + P(n, -1, y - 2 * x - 3) + 2) >> 2;
                break; }
            case 6: {
                int z = 2 * y - x;
                if (z >= 0 && (z & 1) == 0) v = (P(n, -1, y - (x >> 1) - 1) + P(n, -1, y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (P(n, -1, y - (x >> 1) - 2) + 2 * P(n, -1, y - (x >> 1) - 1) + P(n, -1, y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (P(n, -1, 0) + 2 * P(n, -1, -1) + P(n, 0, -1) + 2) >> 2;
                else v = (P(n, x - 2 * y - 1, -1) + 2 * P(n, x - 2 * y - 2, -1) + P(n, x - 2 * y - 3, -1) + 2) >> 2;
                break; }
            case 7:
                if ((y & 1) == 0) v = (P(n, x + (y >> 1), -1) + P(n, x + (y >> 1) + 1, -1) + 1) >> 1;
                else v = (P(n, x + (y >> 1), -1) + 2 * P(n, x + (y >> 1) + 1, -1) + P(n, x + (y >> 1) + 2, -1) + 2) >> 2;
                break;
            default: {
                int z = x + 2 * y;
                if (z < 13 && (z & 1) == 0) v = (P(n, -1, y + (x >> 1)) + P(n, -1, y + (x >> 1) + 1) + 1) >> 1;
                else if (z < 13) v = (P(n, -1, y + (x >> 1)) + 2 * P(n, -1, y + (x >> 1) + 1) + P(n, -1, y + (x >> 1) + 2) + 2) >> 2;
                else if (z == 13) v = (P(n, -1, 6) + 3 * P(n, -1, 7) + 2) >> 2;
                else v = P(n, -1, 7);
                break; }
            }
            pred[yO + y][xO + x] = v;
        }
}

/* Intra16x16 ctor + modes (intra_prediction.cc:624-735); chroma=1: Chroma (:748-894), 4:2:0. */
static void pred_mb(const pstate* s, int addr, int chroma, int mode, const uint8_t* img, int pitch, int pred[16][16])
{
    int N = chroma ? s->MHc : 16;         /* rows (MbHeightC); the width is 8 for chroma */
    int NW = chroma ? 8 : 16;
    int cip = s->p->pic->constrained_intra_pred;
    nbr_t nb, *n = &nb;
    n->stride = 18;
    int nA[16], ax[16], ay[16], bx = 0, by = 0, dx = 0, dy = 0;
    for (int i = 0; i < N; ++i) nA[i] = get_neighbour(s, chroma, addr, -1, i, &ax[i], &ay[i]);
    int nB = get_neighbour(s, chroma, addr, 0, -1, &bx, &by);
    int nD = get_neighbour(s, chroma, addr, -1, -1, &dx, &dy);
    int av[4];
    if (cip) {
        if (!chroma) {
            av[0] = 1;
            for (int i = 0; i < 16; ++i) av[0] &= nA[i] >= 0 && is_intra(s, nA[i]);
            av[2] = 0;
        } else {
            av[0] = 1; av[2] = 1;
            for (int i = 0; i < N / 2; ++i) av[0] &= nA[i] >= 0 && is_intra(s, nA[i]);
            for (int i = N / 2; i < N; ++i) av[2] &= nA[i] >= 0 && is_intra(s, nA[i]);
        }
        av[1] = nB >= 0 && is_intra(s, nB);
        av[3] = nD >= 0 && is_intra(s, nD);
    } else {
        av[0] = nA[0] >= 0; av[1] = nB >= 0;
        av[2] = chroma ? nA[0] >= 0 : 0;
        av[3] = nD >= 0;
    }
    if (av[3]) P(n, -1, -1) = img[dy * pitch + dx];
    if (!chroma) {
        if (av[0]) for (int y = 0; y < 16; ++y) P(n, -1, y) = img[ay[y] * pitch + ax[y]];
    } else {
        if (av[0]) for (int y = 0; y < N / 2; ++y) P(n, -1, y) = img[ay[y] * pitch + ax[y]];
        if (av[2]) for (int y = N / 2; y < N; ++y) P(n, -1, y) = img[ay[y] * pitch + ax[y]];
    }
    if (av[1]) for (int x = 0; x < NW; ++x) P(n, x, -1) = img[by * pitch + bx + x];

    if (!chroma) {
        switch (mode) {
        case 0: for (int y = 0; y < 16; ++y) for (int x = 0; x < 16; ++x) pred[y][x] = P(n, x, -1); break;
        case 1: for (int y = 0; y < 16; ++y) for (int x = 0; x < 16; ++x) pred[y][x] = P(n, -1, y); break;
        case 2: {
            int sum = 0, v;
            if (av[0] || av[1]) {
                if (av[0]) for (int k = 0; k < 16; ++k) sum += P(n, -1, k);
                if (av[1]) for (int k = 0; k < 16; ++k) sum += P(n, k, -1);
                v = (sum + (av[0] ? 8 : 0) + (av[1] ? 8 : 0)) >> (3 + av[0] + av[1]);
            } else v = 128;
            for (int y = 0; y < 16; ++y) for (int x = 0; x < 16; ++x) pred[y][x] = v;
            break; }
        default: {
            int H = 0, V = 0;
            for (int x = 0; x < 8; ++x) H += (x + 1) * (P(n, 8 + x, -1) - P(n, 6 - x, -1));
            for (int y = 0; y < 8; ++y) V += (y + 1) * (P(n, -1, 8 + y) - P(n, -1, 6 - y));
            int a = 16 * (P(n, -1, 15) + P(n, 15, -1));
            int b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) pred[y][x] = clip3(0, 255, (a + b * (x - 7) + c * (y - 7) + 16) >> 5);
            break; }
        }
    } else {
        switch (mode) {
        case 0: /* DC per 4x4 (intra_prediction.cc:825-849), 2 x N/4 blocks */
            for (int blk = 0; blk < N / 2; ++blk) {
                int xO = (blk & 1) * 4, yO = (blk >> 1) * 4;
                int aA, aB;
                if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) { aA = yO > 0 ? av[2] : av[0]; aB = av[1]; }
                else if (xO > 0 && yO == 0) { aA = av[1] ? 0 : av[0]; aB = av[1]; }
                else { aA = av[2]; aB = av[2] ? 0 : av[1]; }
                int sum = 0, v;
                if (aA || aB) {
                    if (aA) for (int k = 0; k < 4; ++k) sum += P(n, -1, k + yO);
                    if (aB) for (int k = 0; k < 4; ++k) sum += P(n, k + xO, -1);
                    v = (sum + (aA ? 2 : 0) + (aB ? 2 : 0)) >> (1 + aA + aB);
                } else v = 128;
                for (int y = 0; y < 4; ++y) for (int x = 0; x < 4; ++x) pred[yO + y][xO + x] = v;
            }
            break;
        case 1: for (int y = 0; y < N; ++y) for (int x = 0; x < 8; ++x) pred[y][x] = P(n, -1, y); break;
        case 2: for (int y = 0; y < N; ++y) for (int x = 0; x < 8; ++x) pred[y][x] = P(n, x, -1); break;
        default: {   /* plane (:871-894): xCF 0, yCF 4 when ChromaArrayType != 1 */
            const int yCF = N == 16 ? 4 : 0;
            int H = 0, V = 0;
            for (int x = 0; x < 4; ++x) H += (x + 1) * (P(n, 4 + x, -1) - P(n, 2 - x, -1));
            for (int y = 0; y < 4 + yCF; ++y) V += (y + 1) * (P(n, -1, 4 + yCF + y) - P(n, -1, 2 + yCF - y));
            int a = 16 * (P(n, -1, N - 1) + P(n, 7, -1));
            int b = (34 * H + 32) >> 6, c = ((yCF ? 5 : 34) * V + 32) >> 6;
            for (int y = 0; y < N; ++y)
                for (int x = 0; x < 8; ++x) pred[y][x] = clip3(0, 255, (a + b * (x - 3) + c * (y - 3 - yCF) + 16) >> 5);
            break; }
        }
    }
}

/* --------------------------------------------------------- inter prediction */
/* pitch: W for a frame; 2 W for a field of a DPB frame (img at the field's first row): the
   reference's split field (dpb_split_field picture.cc:408-470) holds exactly those rows */
static inline int px(const uint8_t* img, int W, int pitch, int H, int x, int y)
{
    return img[clip3(0, H - 1, y) * pitch + clip3(0, W - 1, x)];
}
static inline int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

/* One luma sample of get_block_luma (inter_prediction.cc:158-340), spec 8.4.2.2.1 form. */
static int luma_sample(const uint8_t* img, int W, int pitch, int H, int x, int y, int xf, int yf)
{
#define S(dx, dy) px(img, W, pitch, H, x + (dx), y + (dy))
#define B1(dy) tap6(S(-2, dy), S(-1, dy), S(0, dy), S(1, dy), S(2, dy), S(3, dy))
#define H1(dx) tap6(S(dx, -2), S(dx, -1), S(dx, 0), S(dx, 1), S(dx, 2), S(dx, 3))
    if (xf == 0 && yf == 0) return S(0, 0);
    int b = clip1(255, (B1(0) + 16) >> 5);
    int h = clip1(255, (H1(0) + 16) >> 5);
    if (yf == 0) return xf == 2 ? b : (S(xf == 1 ? 0 : 1, 0) + b + 1) >> 1;
    if (xf == 0) return yf == 2 ? h : (S(0, yf == 1 ? 0 : 1) + h + 1) >> 1;
    if ((xf & 1) && (yf & 1)) {
        int bb = yf == 3 ? clip1(255, (B1(1) + 16) >> 5) : b;
        int hh = xf == 3 ? clip1(255, (H1(1) + 16) >> 5) : h;
        return (bb + hh + 1) >> 1;
    }
    int j1 = tap6(B1(-2), B1(-1), B1(0), B1(1), B1(2), B1(3));
    int j = clip1(255, (j1 + 512) >> 10);
    if (xf == 2 && yf == 2) return j;
    if (xf == 2) { int q0 = yf == 3 ? clip1(255, (B1(1) + 16) >> 5) : b; return (j + q0 + 1) >> 1; }
    { int q0 = xf == 3 ? clip1(255, (H1(1) + 16) >> 5) : h; return (j + q0 + 1) >> 1; }
#undef S
#undef B1
#undef H1
}

/* get_block_chroma sample (inter_prediction.cc:380-404), 4:2:0 frame. */
static int chroma_sample(const uint8_t* img, int W, int pitch, int H, int xi, int yi, int xf, int yf)
{
    int A = px(img, W, pitch, H, xi, yi), B = px(img, W, pitch, H, xi + 1, yi);
    int C = px(img, W, pitch, H, xi, yi + 1), D = px(img, W, pitch, H, xi + 1, yi + 1);
    return ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6;
}

static inline int rshift_rnd(int x, int a) { return a > 0 ? (x + (1 << (a - 1))) >> a : x * (1 << -a); } /* inter_prediction.cc:35-38 */

/* mb_pred_inter + inter_pred + mc_prediction/bi_prediction (decoder.cc:217-262,
 * inter_prediction.cc:53-156, 448-536) into mb_pred[3][16][16]. */
static int inter_pred_mb(const pstate* s, int addr, int mbp[3][16][16])
{
    const oracle_picture* p = s->p;
    const h264r_mb* mb = mb_at(s, addr);
    const h264r_slice* sl = slice_of(s, mb);
    int mbx = addr % s->wmb, mby = addr / s->wmb;
    int plane_n = s->W4 * s->H4;
    /* an MBAFF field MB predicts from fields (get_ref_pic dpb.cc:1046-1055): field refIdx r is frame
       r / 2 of the list, the MB's own parity when r is even; its block rows are field rows
       (block_y_aff, inter_prediction.cc:470-474) of a field of half the height (:172,181-183) */
    const int fmb = s->mbaff && is_field_mb(s, addr), mbot = mby & 1;
    const int fld = s->fld || fmb, cbot = s->fld ? s->bot : mbot;
    const int row4 = fmb ? (mby >> 1) * 4 : mby * 4;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            int idx = (mby * 4 + j) * s->W4 + mbx * 4 + i;
            int r[2], vx[2], vy[2], slot[2], bot[2], vyc[2], rw[2];
            for (int l = 0; l < 2; ++l) {
                r[l] = p->ref_idx[l * plane_n + idx];
                uint32_t m = p->mv[l * plane_n + idx];
                vx[l] = (mbx * 4 + i) * 16 + (int16_t)(m & 0xFFFF);
                vy[l] = (row4 + j) * 16 + (int16_t)(m >> 16);
                rw[l] = fmb && r[l] >= 0 ? r[l] >> 1 : r[l];       /* the weights' index (:66,100-101) */
                int ref = r[l] >= 0 ? sl->ref_slot[l][rw[l]] : -1;
                /* a field picture's list entries name a field of a DPB frame (include/h264r.h) */
                slot[l] = ref < 0 ? -1 : s->fld ? (ref & ~H264R_REF_BOTTOM) : ref;
                bot[l] = s->fld ? ref >= 0 && (ref & H264R_REF_BOTTOM) : fmb && r[l] >= 0 && ((r[l] & 1) != mbot);
                /* get_block_chroma inter_prediction.cc:352-361: a reference field of the other
                   parity moves the chroma vector by -2 (top field / top MB) / +2 (bottom) */
                vyc[l] = vy[l] + (fld && r[l] >= 0 && bot[l] != cbot ? (cbot ? 2 : -2) : 0);
            }
            int dir = (r[0] >= 0 && r[1] >= 0) ? 2 : (r[0] >= 0 ? 0 : (r[1] >= 0 ? 1 : -1));
            if (dir < 0) return H264R_EINVAL;
            for (int l = 0; l < 2; ++l)
                if ((dir == 2 || dir == l) && (slot[l] < 0 || slot[l] >= H264R_MAX_SLOTS || !p->ref_planes[slot[l]][0]))
                    return H264R_EINVAL;
            for (int pl = 0; pl < 3; ++pl) {
                /* the 4x4 block's chroma: 2 x 2 (4:2:0) or 2 x 4 (4:2:2) samples */
                int nw = pl ? 2 : 4, nh = pl ? s->MHc / 4 : 4, ox = pl ? i * 2 : i * 4, oy = j * nh;
                int Wp = pl ? s->Wc : s->W, Hp = pl ? s->Hc : s->H;
                for (int y = 0; y < nh; ++y)
                    for (int x = 0; x < nw; ++x) {
                        int v[2] = {0, 0};
                        for (int l = 0; l < 2; ++l) {
                            if (!(dir == 2 || dir == l)) continue;
                            const uint8_t* img = p->ref_planes[slot[l]][pl] + bot[l] * Wp;
                            const int pitch = Wp << fld, Hv = fmb ? Hp >> 1 : Hp;
                            if (!pl) v[l] = luma_sample(img, Wp, pitch, Hv, (vx[l] >> 2) + x, (vy[l] >> 2) + y, vx[l] & 3, vy[l] & 3);
                            else if (s->cf == 1) v[l] = chroma_sample(img, Wp, pitch, Hv, (vx[l] >> 3) + x, (vyc[l] >> 3) + y, vx[l] & 7, vyc[l] & 7);
                            else v[l] = chroma_sample(img, Wp, pitch, Hp, (vx[l] >> 3) + x, (vy[l] >> 2) + y, vx[l] & 7,
                                                      (vy[l] & 3) << 1);   /* 4:2:2: yAL = mv >> 2, yFracC (mv & 3) << 1 (:381-383) */
                        }
                        int out;
                        if (dir != 2) {
                            int wpf = sl->wp_mode == 1;      /* mc_prediction :62-85 */
                            if (wpf) {
                                int w = sl->wp_weight[dir][rw[dir]][pl], o = sl->wp_offset[dir][rw[dir]][pl];
                                int d = pl ? sl->chroma_log2_wd : sl->luma_log2_wd;
                                out = clip1(255, rshift_rnd(w * v[dir], d) + o);
                            } else out = v[dir];
                        } else if (sl->wp_mode) {               /* bi_prediction :99-153 */
                            int w0, w1, o0, o1;
                            if (sl->wp_mode == 1) {
                                w0 = sl->wp_weight[0][rw[0]][pl]; w1 = sl->wp_weight[1][rw[1]][pl];
                                o0 = sl->wp_offset[0][rw[0]][pl]; o1 = sl->wp_offset[1][rw[1]][pl];
                            } else {
                                if (fmb) return H264R_EUNSUPPORTED;      /* field-MB implicit weights: not on the path */
                                w1 = sl->implicit_w1[r[0]][r[1]]; w0 = 64 - w1; o0 = o1 = 0;
                            }
                            int d = (pl ? sl->chroma_log2_wd : sl->luma_log2_wd) + 1;
                            out = clip1(255, rshift_rnd(w0 * v[0] + w1 * v[1], d) + ((o0 + o1 + 1) >> 1));
                        } else out = (v[0] + v[1] + 1) >> 1;
                        mbp[pl][oy + y][ox + x] = out;
                    }
            }
        }
    return 0;
}

/* ------------------------------------------------------------ construction */
static uint8_t* plane_ptr(const pstate* s, int pl) { return s->p->out[pl]; }

/* construction / construction_16x16 / construction_chroma (transform.cc:913-984) */
static void construct(const pstate* s, int addr, int pl, int x0, int y0, int w, int h,
                      int use_res, int rres[16][16], int mbp[16][16])
{
    int mbx = addr % s->wmb, mby = addr / s->wmb;
    int NW = pl ? 8 : 16, NH = pl ? s->MHc : 16, pitch = pl ? s->Wc : s->W;
    uint8_t* img = plane_ptr(s, pl) + (mby * NH) * pitch + mbx * NW;
    for (int y = y0; y < y0 + h; ++y) {
        uint8_t* row = img + y * pitch;
        if (s->mbaff) { int gx, gy; mbaff_loc(s, addr, NW, NH, 0, y, &gx, &gy); row = plane_ptr(s, pl) + gy * pitch + gx; }
        for (int x = x0; x < x0 + w; ++x)
            row[x] = (uint8_t)(use_res ? clip1(255, rres[y][x] + mbp[y][x]) : mbp[y][x]);
    }
}

static int intra4_mode(const h264r_mb* mb, int blk) { return (mb->ipred[blk >> 1] >> ((blk & 1) * 4)) & 15; }

/* inverse_transform_4x4 / _8x8 of one coded block (transform.cc:986-1016): the inverse
 * transform, or for TransformBypassModeFlag MBs the DPCM of the block's Intra4x4PredMode /
 * Intra8x8PredMode (read for inter MBs too, :993,1008). */
static void luma_block_res(const h264r_mb* mb, int cof[16][16], int rres[16][16], int x, int y, int n)
{
    int bk = n == 4 ? ((y / 4) / 2) * 8 + ((y / 4) % 2) * 2 + ((x / 4) / 2) * 4 + ((x / 4) % 2)
                    : (y / 8) * 2 + x / 8;
    if (mb->flags & H264R_MBF_BYPASS) bypass_block(cof, rres, x, y, n, n, intra4_mode(mb, bk), 0, 1);
    else if (n == 4) inverse_4x4(cof, rres, y, x);
    else inverse_8x8(cof, rres, y, x);
}

/* inverse_transform_16x16 / inverse_transform_chroma residual (transform.cc:1018-1049) */
static void mb_res(const pstate* s, const h264r_mb* mb, int pl, int cof[16][16], int rres[16][16])
{
    int nw = pl ? 8 : 16, nh = pl ? s->MHc : 16;
    if (mb->flags & H264R_MBF_BYPASS)
        bypass_block(cof, rres, 0, 0, nw, nh, pl ? mb->chroma_mode : mb->i16_mode, pl ? 2 : 0, 1);
    else
        for (int y = 0; y < nh; y += 4) for (int x = 0; x < nw; x += 4) inverse_4x4(cof, rres, y, x);
}

/* ------------------------------------------------------- SP slices (transform.cc:1098-1300) */
static const int A_SP[4][4] = {{16, 20, 16, 20}, {20, 25, 20, 25}, {16, 20, 16, 20}, {20, 25, 20, 25}};   /* :1098-1103 */

/* LevelScale2 (transform.cc:1105-1130): the forward quantisation scale, by position class */
static int level_scale2(int m, int j, int i)
{
    static const int v[6][3] = {{13107, 8066, 5243}, {11916, 7490, 4660}, {10082, 6554, 4194},
                                {9362, 5825, 3647}, {8192, 5243, 3355}, {7282, 4559, 2893}};
    return v[m][(j & 1) + (i & 1)];
}

static inline int sgn(int x) { return (x >= 0) - (x < 0); }                          /* defines.h:73-77 */
static inline int shl(int x, int s) { return (int)((unsigned)x << s); }              /* C++ << on negatives */

static void forward_4x4(int p[16][16], int c[16][16], int py, int px)               /* transform.cc:556-595 */
{
    int f[4][4];
    for (int i = 0; i < 4; ++i) {
        int e0 = p[py + i][px + 0] + p[py + i][px + 3], e1 = p[py + i][px + 1] + p[py + i][px + 2];
        int e2 = p[py + i][px + 1] - p[py + i][px + 2], e3 = p[py + i][px + 0] - p[py + i][px + 3];
        f[i][0] = e0 + e1; f[i][1] = e2 + (e3 << 1); f[i][2] = e0 - e1; f[i][3] = e3 - (e2 << 1);
    }
    for (int j = 0; j < 4; ++j) {
        int g0 = f[0][j] + f[3][j], g1 = f[1][j] + f[2][j], g2 = f[1][j] - f[2][j], g3 = f[0][j] - f[3][j];
        c[py + 0][px + j] = g0 + g1; c[py + 1][px + j] = g2 + (g3 << 1);
        c[py + 2][px + j] = g0 - g1; c[py + 3][px + j] = g3 - (g2 << 1);
    }
}

/* An inter MB of an SP slice: Transform::inverse_transform_sp (transform.cc:1267-1300) --
 * itrans_sp per luma 4x4 block (:1132-1187; reconstruction = clip1 of the residual, the
 * prediction enters in the transform domain), then per chroma plane itrans_sp_cr
 * (:1190-1265) and inverse_transform_chroma (which adds the prediction once more, as the
 * reference does: itrans_sp_cr keeps mb_pred, :1209).  cof holds what the coefficient push
 * left: dequantised AC levels and, chroma DC, the raw levels (transform_chroma_dc skips SP
 * inter MBs, :865-875).  Luma QP: the MB's QpY (slice.parser.QpY at decode time). */
static void sp_mb(const pstate* s, int addr, const h264r_mb* mb, int cof[3][16][16], int mbp[3][16][16])
{
    const h264r_slice* sl = slice_of(s, mb);
    static __thread int c[16][16], rres[16][16];
    const int sw = sl->sp_switch;
    {
        const int qp = mb->qp_y, qs = sl->qs_y;
        for (int by = 0; by < 16; by += 4)
            for (int bx = 0; bx < 16; bx += 4) {
                forward_4x4(mbp[0], c, by, bx);
                for (int j = 0; j < 4; ++j)
                    for (int i = 0; i < 4; ++i) {
                        int crij = cof[0][by + j][bx + i], cpij = c[by + j][bx + i], cij;
                        int ls = level_scale2(qs % 6, j, i);
                        if (sw) {
                            int csij = sgn(cpij) * ((iabs(cpij) * ls + (1 << (14 + qs / 6))) >> (15 + qs / 6));
                            cij = crij + csij;
                        } else {
                            int csij = cpij + (shl(crij * dequant_coef[qp % 6][j][i] * A_SP[j][i], qp / 6) >> 10);
                            cij = sgn(csij) * ((iabs(csij) * ls + (1 << (14 + qs / 6))) >> (15 + qs / 6));
                        }
                        int dq = dequant_coef[qs % 6][j][i];
                        cof[0][by + j][bx + i] = qs >= 24 ? shl(cij * dq, qs / 6 - 4) : (cij * dq + (1 << (3 - qs / 6))) >> (4 - qs / 6);
                    }
                inverse_4x4(cof[0], rres, by, bx);
                for (int j = 0; j < 4; ++j)
                    for (int i = 0; i < 4; ++i) mbp[0][by + j][bx + i] = clip1(255, rres[by + j][bx + i]);
            }
        construct(s, addr, 0, 0, 0, 16, 16, 0, rres, mbp[0]);      /* the reconstruction itself */
    }
    levels_view v = view_levels(mb, s->p->levels, 1);
    for (int pl = 1; pl <= 2; ++pl) {
        const int qp = mb->qp_c[pl - 1], qs = sl->qs_c[pl - 1];     /* QsC < 6 (see h264r_synth.h) */
        int (*cf)[16] = cof[pl];
        for (int n2 = 0; n2 < 2; ++n2)                              /* raw DC levels */
            for (int n1 = 0; n1 < 2; ++n1) cf[n2 * 4][n1 * 4] = v.cdc ? v.cdc[(pl - 1) * 4 + n2 * 2 + n1] : 0;
        for (int y = 0; y < 8; y += 4) for (int x = 0; x < 8; x += 4) forward_4x4(mbp[pl], c, y, x);
        int mp1[2][2];
        mp1[0][0] = c[0][0] + c[4][0] + c[0][4] + c[4][4];
        mp1[0][1] = c[0][0] - c[4][0] + c[0][4] - c[4][4];
        mp1[1][0] = c[0][0] + c[4][0] - c[0][4] - c[4][4];
        mp1[1][1] = c[0][0] - c[4][0] - c[0][4] + c[4][4];
        for (int n2 = 0; n2 < 2; ++n2)
            for (int n1 = 0; n1 < 2; ++n1) {
                int crij = cf[n2 * 4][n1 * 4], cpij = mp1[n2][n1], cij;
                int ls = level_scale2(qs % 6, 0, 0);
                if (sw) {
                    int csij = (sgn(cpij) * (iabs(cpij) * ls + (1 << (15 + qs / 6)))) >> (16 + qs / 6);
                    cij = csij + cpij;
                } else {
                    int csij = cpij + (shl(crij * dequant_coef[qp % 6][0][0] * A_SP[0][0], qp / 6) >> 9);
                    cij = (sgn(csij) * (iabs(csij) * ls + (1 << (15 + qs / 6)))) >> (16 + qs / 6);
                }
                mp1[n2][n1] = shl(cij * dequant_coef[qs % 6][0][0], qp / 6);
            }
        for (int n2 = 0; n2 < 8; n2 += 4)
            for (int n1 = 0; n1 < 8; n1 += 4)
                for (int j = 0; j < 4; ++j)
                    for (int i = 0; i < 4; ++i) {
                        /* the prediction SAMPLE, not its transform (transform.cc:1246) */
                        int crij = cf[n2 + j][n1 + i], cpij = mbp[pl][n2 + j][n1 + i], cij;
                        int ls = level_scale2(qs % 6, j, i);
                        if (sw) {
                            int csij = (sgn(cpij) * (iabs(cpij) * ls + (1 << (14 + qs / 6)))) >> (15 + qs / 6);
                            cij = crij + csij;
                        } else {
                            int csij = cpij + (shl(crij * dequant_coef[qp % 6][j][i] * A_SP[j][i], qp / 6) >> 9);
                            cij = (sgn(csij) * (iabs(csij) * ls + (1 << (14 + qs / 6)))) >> (15 + qs / 6);
                        }
                        cf[n2 + j][n1 + i] = shl(cij * dequant_coef[qs % 6][j][i], qp / 6);
                    }
        cf[0][0] = (mp1[0][0] + mp1[0][1] + mp1[1][0] + mp1[1][1]) >> 1;
        cf[0][4] = (mp1[0][0] + mp1[0][1] - mp1[1][0] - mp1[1][1]) >> 1;
        cf[4][0] = (mp1[0][0] - mp1[0][1] + mp1[1][0] - mp1[1][1]) >> 1;
        cf[4][4] = (mp1[0][0] - mp1[0][1] - mp1[1][0] + mp1[1][1]) >> 1;
        for (int y = 0; y < 8; y += 4) for (int x = 0; x < 8; x += 4) inverse_4x4(cf, rres, y, x);
        construct(s, addr, pl, 0, 0, 8, 8, 1, rres, mbp[pl]);
    }
}

/* Decoder::decode (decoder.cc:65-262) for one MB. */
static int decode_mb(pstate* s, int addr)
{
    const oracle_picture* p = s->p;
    const h264r_mb* mb = mb_at(s, addr);
    int mbx = addr % s->wmb, mby = addr / s->wmb;
    static __thread int cof[3][16][16], rres[3][16][16], mbp[3][16][16];
    s->slice_nr[addr] = (int16_t)mb->slice;               /* mb.init, slice_data.cc:465 */
    if (s->mbaff && ((mb->flags & H264R_MBF_BYPASS) || slice_of(s, mb)->slice_type >= H264R_SLICE_SP))
        return H264R_EUNSUPPORTED;                        /* lossless / SP MBAFF: not on the path */

    if (mb->mb_type == H264R_I_PCM) {                      /* mb_pred_ipcm decoder.cc:149-168 */
        const uint8_t* raw = (const uint8_t*)(p->levels + mb->coef_off);
        for (int y = 0; y < 16; ++y) for (int x = 0; x < 16; ++x) mbp[0][y][x] = raw[y * 16 + x];
        for (int k = 0; k < 2; ++k)
            for (int y = 0; y < s->MHc; ++y) for (int x = 0; x < 8; ++x) mbp[1 + k][y][x] = raw[256 + k * 8 * s->MHc + y * 8 + x];
        for (int pl = 0; pl < 3; ++pl) construct(s, addr, pl, 0, 0, pl ? 8 : 16, pl ? s->MHc : 16, 0, rres[pl], mbp[pl]);
        (void)mbx; (void)mby;
        return 0;
    }
    load_cof(mb, p->levels, p->quant, s->cf, cof);
    int cbpl = mb->cbp & 15, cbpc = mb->cbp >> 4;

    if (mb->mb_type == H264R_I_4x4 || mb->mb_type == H264R_I_8x8 || mb->mb_type == H264R_I_16x16) {
        /* mb_pred_intra decoder.cc:170-208 */
        const uint8_t* img = p->out[0];
        int step = mb->mb_type == H264R_I_4x4 ? 1 : mb->mb_type == H264R_I_8x8 ? 4 : 16;
        for (int b = 0; b < 16; b += step) {
            int ioff = ((b / 4) % 2) * 8 + ((b % 4) % 2) * 4;
            int joff = ((b / 4) / 2) * 8 + ((b % 4) / 2) * 4;
            if (mb->mb_type == H264R_I_4x4) {
                nbr_t n;
                gather_nxn(s, addr, 4, ioff, joff, img, s->W, &n);
                pred_4x4(&n, intra4_mode(mb, b), mbp[0], ioff, joff);
                int coded = cbpl & (1 << ((joff / 8) * 2 + ioff / 8));
                if (coded) luma_block_res(mb, cof[0], rres[0], ioff, joff, 4);
                construct(s, addr, 0, ioff, joff, 4, 4, coded, rres[0], mbp[0]);
            } else if (mb->mb_type == H264R_I_8x8) {
                nbr_t n, f;
                gather_nxn(s, addr, 8, ioff, joff, img, s->W, &n);
                filter_8x8(&n, &f);
                pred_8x8(&f, intra4_mode(mb, b / 4), mbp[0], ioff, joff);
                int coded = cbpl & (1 << ((joff / 8) * 2 + ioff / 8));
                if (coded) luma_block_res(mb, cof[0], rres[0], ioff, joff, 8);
                construct(s, addr, 0, ioff, joff, 8, 8, coded, rres[0], mbp[0]);
            } else {
                pred_mb(s, addr, 0, mb->i16_mode, img, s->W, mbp[0]);
                mb_res(s, mb, 0, cof[0], rres[0]);
                construct(s, addr, 0, 0, 0, 16, 16, 1, rres[0], mbp[0]);
            }
        }
        for (int pl = 1; pl <= 2; ++pl) {
            pred_mb(s, addr, 1, mb->chroma_mode, p->out[pl], s->Wc, mbp[pl]);
        }
        for (int pl = 1; pl <= 2; ++pl) {                  /* inverse_transform_chroma :1033-1049 */
            mb_res(s, mb, pl, cof[pl], rres[pl]);
            construct(s, addr, pl, 0, 0, 8, s->MHc, 1, rres[pl], mbp[pl]);
        }
        return 0;
    }

    int st = inter_pred_mb(s, addr, mbp);
    if (st) return st;
    if (slice_of(s, mb)->slice_type == H264R_SLICE_SP) {          /* decoder.cc:256-257 */
        if (mb->flags & H264R_MBF_T8x8) return H264R_EUNSUPPORTED;  /* no 8x8 transform in SP (Extended) */
        if (s->cf != 1) return H264R_EUNSUPPORTED;                  /* nor 4:2:2 (Extended is 4:2:0) */
        sp_mb(s, addr, mb, cof, mbp);
        return 0;
    }
    /* inverse_transform_inter transform.cc:1051-1095 */
    if (cbpl) {
        if (!(mb->flags & H264R_MBF_T8x8)) {
            for (int y = 0; y < 16; y += 4)
                for (int x = 0; x < 16; x += 4) {
                    int coded = cbpl & (1 << ((y / 8) * 2 + x / 8));
                    if (coded) luma_block_res(mb, cof[0], rres[0], x, y, 4);
                    construct(s, addr, 0, x, y, 4, 4, coded, rres[0], mbp[0]);
                }
        } else {
            for (int y = 0; y < 16; y += 8)
                for (int x = 0; x < 16; x += 8) {
                    int coded = cbpl & (1 << ((y / 8) * 2 + x / 8));
                    if (coded) luma_block_res(mb, cof[0], rres[0], x, y, 8);
                    construct(s, addr, 0, x, y, 8, 8, coded, rres[0], mbp[0]);
                }
        }
    } else construct(s, addr, 0, 0, 0, 16, 16, 0, rres[0], mbp[0]);
    for (int pl = 1; pl <= 2; ++pl) {
        if (cbpc) {
            mb_res(s, mb, pl, cof[pl], rres[pl]);
            construct(s, addr, pl, 0, 0, 8, s->MHc, 1, rres[pl], mbp[pl]);
        } else construct(s, addr, pl, 0, 0, 8, s->MHc, 0, rres[pl], mbp[pl]);
    }
    return 0;
}

/* ---------------------------------------------------------------- deblocking */
static const uint8_t TABLE_ALPHA[52] = {                               /* deblock.cc:294-299 */
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10, 12, 13,
    15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static const uint8_t TABLE_BETA[52] = {                                /* deblock.cc:301-306 */
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4,
    6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static const uint8_t TABLE_TC0[52][3] = {                              /* deblock.cc:310-324 */
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1},
    {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3},
    {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6},
    {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16},
    {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

typedef struct { int ref[2]; int mvx[2], mvy[2]; } mvinfo_t;

/* pic_motion_params of one 4x4 block; ref = DPB slot identity (ref_pic pointer) or -1. */
static mvinfo_t mvinfo(const pstate* s, int bx4, int by4)
{
    const oracle_picture* p = s->p;
    int plane_n = s->W4 * s->H4, idx = by4 * s->W4 + bx4;
    const int addr = (by4 / 4) * s->wmb + bx4 / 4;
    const h264r_mb* mb = mb_at(s, addr);
    const h264r_slice* sl = slice_of(s, mb);
    /* an MBAFF field MB's pictures are fields (get_ref_pic dpb.cc:1046-1055): slot | 0x80, with
       H264R_REF_BOTTOM for the bottom field, never equal to the frame's identity */
    const int fmb = s->mbaff && is_field_mb(s, addr), mbot = (addr / s->wmb) & 1;
    mvinfo_t m;
    for (int l = 0; l < 2; ++l) {
        int r = p->ref_idx[l * plane_n + idx];
        uint32_t v = p->mv[l * plane_n + idx];
        m.ref[l] = r < 0 ? -1 : !fmb ? sl->ref_slot[l][r]
                 : (sl->ref_slot[l][r >> 1] | 0x80 | (((r & 1) != mbot) ? H264R_REF_BOTTOM : 0));
        m.mvx[l] = (int16_t)(v & 0xFFFF);
        m.mvy[l] = (int16_t)(v >> 16);
    }
    return m;
}

/* deblock.cc:35-38; mvlimit = 2 in field pictures, 4 in frames (deblock.cc:86,164) */
static inline int compare_mvs(const mvinfo_t* a, int la, const mvinfo_t* b, int lb, int mvlimit)
{
    return (iabs(a->mvx[la] - b->mvx[lb]) >= 4) | (iabs(a->mvy[la] - b->mvy[lb]) >= mvlimit);
}

/* deblock.cc:40-75; ref identity: the DPB slot with the field parity bit (the two fields of a
   frame are different storable_pictures in the reference) */
static int bs_compare_mvs(const mvinfo_t* p, const mvinfo_t* q, int ml)
{
    int p0 = p->ref[0], q0 = q->ref[0], p1 = p->ref[1], q1 = q->ref[1];
    if ((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0)) {
        if (p0 != p1) {
            if (p0 == q0) return compare_mvs(p, 0, q, 0, ml) | compare_mvs(p, 1, q, 1, ml);
            return compare_mvs(p, 0, q, 1, ml) | compare_mvs(p, 1, q, 0, ml);
        }
        return (compare_mvs(p, 0, q, 0, ml) | compare_mvs(p, 1, q, 1, ml)) &
               (compare_mvs(p, 0, q, 1, ml) | compare_mvs(p, 1, q, 0, ml));
    }
    return 1;
}

static int is_special(const pstate* s, const h264r_mb* m)
{
    int t = slice_of(s, m)->slice_type;
    return t == H264R_SLICE_SP || t == H264R_SLICE_SI;
}

/* Deblock::strength + strength_vertical/horizontal (deblock.cc:78-289), frame and field
   pictures (a field picture: mvlimit 2, and cond_bS4 = !field || verticalEdgeFlag,
   deblock.cc:103-107,184-189, so its horizontal MB edges get bS 3 where a frame's get 4). */
static void strength(pstate* s, int addr)
{
    const h264r_mb* q = mb_at(s, addr);
    const h264r_slice* sl = slice_of(s, q);
    int mbx = addr % s->wmb, mby = addr / s->wmb;
    memset(s->fver[addr], 0, sizeof(s->fver[addr]));
    memset(s->fhor[addr], 0, sizeof(s->fhor[addr]));
    if (sl->deblock_idc == 1) return;
    int L = mbx > 0 ? addr - 1 : -1, U = mby > 0 ? addr - s->wmb : -1;
    int fl = 0, ft = 0;
    if (sl->deblock_idc == 0) { fl = L >= 0; ft = U >= 0; }
    else if (sl->deblock_idc == 2) {
        fl = L >= 0 && mb_at(s, L)->slice == q->slice;
        ft = U >= 0 && mb_at(s, U)->slice == q->slice;
    }
    for (int c = 0; c < 2; ++c) {
        s->fver[addr][c][0] = fl; s->fhor[addr][c][0] = ft;
        for (int e = 1; e < 4; ++e) s->fver[addr][c][e] = s->fhor[addr][c][e] = 1;
    }
    if (q->flags & H264R_MBF_T8x8) s->fver[addr][0][1] = s->fver[addr][0][3] = s->fhor[addr][0][1] = s->fhor[addr][0][3] = 0;
    s->fver[addr][1][2] = s->fver[addr][1][3] = 0;
    if (s->cf == 1) s->fhor[addr][1][2] = s->fhor[addr][1][3] = 0;     /* 4:2:2 keeps 4 (:270-275) */

    int qintra = (q->flags & H264R_MBF_INTRA) != 0;
    int pskip = sl->slice_type == H264R_SLICE_P && q->mb_type == H264R_P_SKIP;
    for (int e = 0; e < 4; ++e) {
        if (s->fver[addr][0][e]) {                                  /* strength_vertical */
            uint8_t* St = s->strength_ver[addr][e];
            const h264r_mb* pm = e == 0 ? mb_at(s, L) : q;
            int special = is_special(s, pm) || is_special(s, q);
            if (e == 0 && special) memset(St, 4, 16);
            else if (special) memset(St, 3, 16);
            else if (e > 0 && pskip) memset(St, 0, 16);
            else {
                int intra = qintra || (pm->flags & H264R_MBF_INTRA);
                for (int y = 0; y < 16; ++y) {
                    int v;
                    int blkQ = (y & 12) + e, blkP = (y & 12) + (e == 0 ? 3 : e - 1);
                    if (e == 0 && intra) v = 4;
                    else if (intra) v = 3;
                    else if (((q->cbp_blks >> blkQ) & 1) || ((pm->cbp_blks >> blkP) & 1)) v = 2;
                    else if (e > 0 && (q->mb_type == H264R_P_16x16 || q->mb_type == H264R_P_16x8)) v = 0;
                    else {
                        mvinfo_t mq = mvinfo(s, mbx * 4 + e, mby * 4 + y / 4);
                        mvinfo_t mp = mvinfo(s, mbx * 4 + e - 1, mby * 4 + y / 4);
                        v = bs_compare_mvs(&mq, &mp, s->fld ? 2 : 4);
                    }
                    St[y] = (uint8_t)v;
                }
            }
        }
        /* strength_horizontal.  4:2:2: the chroma edges at rows 4 and 12 read strength_hor[1] / [3]
           (filter_edge :433) also in an MB with transform_size_8x8_flag, whose luma edges 1 and 3
           the reference does not filter and so never computes bS for (:280-285): it reads what the
           mb_t slot last held.  The restatement computes them as JM and 8.7.2.1 do (the same
           derivation at those rows); the golden fixtures keep 4:2:2 pictures free of 8x8
           transforms, where the two agree (tests/golden/make_golden.py). */
        if (s->fhor[addr][0][e] || (s->cf == 2 && s->fhor[addr][1][e])) {
            uint8_t* St = s->strength_hor[addr][e];
            const h264r_mb* pm = e == 0 ? mb_at(s, U) : q;
            int special = is_special(s, pm) || is_special(s, q);
            int intra = qintra || (pm->flags & H264R_MBF_INTRA);
            if (e == 0 && !s->fld && (special || intra)) memset(St, 4, 16);
            else if (special || intra) memset(St, 3, 16);
            else if (e > 0 && pskip) memset(St, 0, 16);
            else {
                for (int x4 = 0; x4 < 4; ++x4) {
                    int v;
                    int blkQ = 4 * e + x4, blkP = (e == 0 ? 12 : 4 * (e - 1)) + x4;
                    if (((q->cbp_blks >> blkQ) & 1) || ((pm->cbp_blks >> blkP) & 1)) v = 2;
                    else if (e > 0 && (q->mb_type == H264R_P_16x16 || q->mb_type == H264R_P_8x16)) v = 0;
                    else {
                        mvinfo_t mq = mvinfo(s, mbx * 4 + x4, mby * 4 + e);
                        mvinfo_t mp = mvinfo(s, mbx * 4 + x4, mby * 4 + e - 1);
                        v = bs_compare_mvs(&mq, &mp, s->fld ? 2 : 4);
                    }
                    memset(St + 4 * x4, v, 4);
                }
            }
        }
    }
}

/* filter_strong / filter_normal (deblock.cc:327-415) on one line across the edge. */
static void filter_line(uint8_t* q, int inc, int alpha, int beta, int bS, int chroma, int tc0)
{
#define Pp(i) q[-((i) + 1) * inc]
#define Qq(i) q[(i) * inc]
    int p0 = Pp(0), p1 = Pp(1), p2 = Pp(2), q0 = Qq(0), q1 = Qq(1), q2 = Qq(2);
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    if (bS == 4) {
        int np0, np1, np2, nq0, nq1, nq2;
        if (!chroma && ap < beta && iabs(p0 - q0) < (alpha >> 2) + 2) {
            int p3 = Pp(3);
            np0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
            np1 = (p2 + p1 + p0 + q0 + 2) >> 2;
            np2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
        } else { np0 = (2 * p1 + p0 + q1 + 2) >> 2; np1 = p1; np2 = p2; }
        if (!chroma && aq < beta && iabs(p0 - q0) < (alpha >> 2) + 2) {
            int q3 = Qq(3);
            nq0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
            nq1 = (p0 + q0 + q1 + q2 + 2) >> 2;
            nq2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
        } else { nq0 = (2 * q1 + q0 + p1 + 2) >> 2; nq1 = q1; nq2 = q2; }
        Pp(0) = (uint8_t)np0; Pp(1) = (uint8_t)np1; Pp(2) = (uint8_t)np2;
        Qq(0) = (uint8_t)nq0; Qq(1) = (uint8_t)nq1; Qq(2) = (uint8_t)nq2;
    } else {
        int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
        int delta = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
        int np1 = p1, nq1 = q1;
        if (!chroma && ap < beta) np1 = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 * 2)) >> 1);
        if (!chroma && aq < beta) nq1 = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 * 2)) >> 1);
        Pp(0) = (uint8_t)clip1(255, p0 + delta);
        Qq(0) = (uint8_t)clip1(255, q0 - delta);
        Pp(1) = (uint8_t)np1; Qq(1) = (uint8_t)nq1;
    }
#undef Pp
#undef Qq
}

/* filter_edge (deblock.cc:418-486), 4:2:0 / 4:2:2.  `edge` is the sample offset. */
static void filter_edge(pstate* s, int addr, int chroma, int pl, int vertical, int edge)
{
    const h264r_mb* q = mb_at(s, addr);
    const h264r_slice* sl = slice_of(s, q);
    int mbx = addr % s->wmb, mby = addr / s->wmb;
    const uint8_t* St = vertical ? s->strength_ver[addr][chroma ? edge * 4 / 8 : edge / 4]
                                 : s->strength_hor[addr][chroma ? edge * 4 / s->MHc : edge / 4];
    int nE = !chroma ? 16 : vertical ? s->MHc : 8;
    int pitch = chroma ? s->Wc : s->W;
    int x0 = mbx * (chroma ? 8 : 16), y0 = mby * (chroma ? s->MHc : 16);
    uint8_t* img = s->p->out[pl];
    int paddr = edge == 0 ? (vertical ? addr - 1 : addr - s->wmb) : addr;
    const h264r_mb* pm = mb_at(s, paddr);
    int qPp = chroma ? pm->qp_c[pl - 1] : pm->qp_y, qPq = chroma ? q->qp_c[pl - 1] : q->qp_y;
    int qPav = (qPp + qPq + 1) >> 1;
    int indexA = clip3(0, 51, qPav + sl->filter_offset_a);
    int indexB = clip3(0, 51, qPav + sl->filter_offset_b);
    int alpha = TABLE_ALPHA[indexA], beta = TABLE_BETA[indexB];
    for (int pel = 0; pel < nE; ++pel) {
        int bS = St[nE == 8 ? pel << 1 : pel];
        if (!bS) continue;
        uint8_t* qp = vertical ? &img[(y0 + pel) * pitch + x0 + edge] : &img[(y0 + edge) * pitch + x0 + pel];
        int inc = vertical ? 1 : pitch;
        filter_line(qp, inc, alpha, beta, bS, chroma, bS < 4 ? TABLE_TC0[indexA][bS - 1] : 0);
    }
}


/* ---- MBAFF frames: Deblock::strength / strength_vertical / strength_horizontal / filter_edge with
   MbaffFrameFlag (deblock.cc:78-289, 418-535), on the frame after MbAffPostProc (:596-629).  Sample
   positions are Neighbour::get_location / get_neighbour's (mbaff_loc / mbaff_mb_at); a block's
   motion sits at the MB's storage row (mv_info[nb.y / 4], nb.y the MB-local row). */
static int mbaff_mvinfo_row(const pstate* s, int n, int ly) { return (n / s->wmb) * 4 + ly / 4; }

static void strength_vertical_mbaff(pstate* s, int addr, int e)          /* deblock.cc:78-155 */
{
    const h264r_mb* q = mb_at(s, addr);
    uint8_t* St = s->strength_ver[addr][e];
    const int fq = is_field_mb(s, addr), mvlimit = fq ? 2 : 4, dy = 1 + fq;
    int xq, yq, lyp;
    mbaff_loc(s, addr, 16, 16, e * 4, 0, &xq, &yq);
    int P = mbaff_mb_at(s, 16, 16, xq - 1, yq, &lyp);
    const h264r_mb* pm = mb_at(s, P);
    const int mixed = fq != is_field_mb(s, P);
    const int special = is_special(s, pm) || is_special(s, q);
    /* cond_bS4 = !field || (MbaffFrameFlag && verticalEdgeFlag) = 1; cond_bS3 = !mixed */
    if (e == 0 && special) { memset(St, 4, 16); return; }
    if (!mixed && special) { memset(St, 3, 16); return; }
    if (e > 0 && slice_of(s, q)->slice_type == H264R_SLICE_P && q->mb_type == H264R_P_SKIP) { memset(St, 0, 16); return; }
    for (int y = 0; y < 16; ++y) {
        int v;
        const int intra = ((pm->flags | q->flags) & H264R_MBF_INTRA) != 0;
        const int blkP = (lyp & 12) + ((xq - 1) & 15) / 4, blkQ = (y & 12) + e;
        if (e == 0 && intra) v = 4;
        else if (!mixed && intra) v = 3;
        else if (((q->cbp_blks >> blkQ) & 1) || ((pm->cbp_blks >> blkP) & 1)) v = 2;
        else if (mixed) v = 1;
        else if (e > 0 && (q->mb_type == H264R_P_16x16 || q->mb_type == H264R_P_16x8)) v = 0;
        else {
            mvinfo_t mq = mvinfo(s, xq / 4, mbaff_mvinfo_row(s, addr, y));
            mvinfo_t mp = mvinfo(s, (xq - 1) / 4, mbaff_mvinfo_row(s, P, lyp));
            v = bs_compare_mvs(&mq, &mp, mvlimit);
        }
        St[y] = (uint8_t)v;
        if (y < 15) { P = mbaff_mb_at(s, 16, 16, xq - 1, yq + dy * (y + 1), &lyp); pm = mb_at(s, P); }
    }
}

static void strength_horizontal_mbaff(pstate* s, int addr, int e)        /* deblock.cc:157-228 */
{
    const h264r_mb* q = mb_at(s, addr);
    uint8_t* St = e == 4 ? s->strength_hor4[addr] : s->strength_hor[addr][e];
    const int fq = is_field_mb(s, addr), mvlimit = fq ? 2 : 4;
    const int dy = 1 + (fq || ((e == 0 || e == 4) && s->fhor4[addr][0]));
    int xq, yq, lyq, lyp;
    mbaff_loc(s, addr, 16, 16, 0, 0, &xq, &yq);
    yq += e == 4 ? 1 : dy * e * 4;
    const int Q = mbaff_mb_at(s, 16, 16, xq, yq, &lyq);
    const int P = mbaff_mb_at(s, 16, 16, xq, yq - dy, &lyp);
    const h264r_mb* pm = mb_at(s, P);
    const int mixed = fq != is_field_mb(s, P);
    const int special = is_special(s, pm) || is_special(s, q);
    const int field = is_field_mb(s, P) || fq;
    const int intra = ((pm->flags | q->flags) & H264R_MBF_INTRA) != 0;
    /* cond_bS4 = !field (horizontal), cond_bS3 = 1 */
    if (e == 0 && !field && (special || intra)) { memset(St, 4, 16); return; }
    if (special || intra) { memset(St, 3, 16); return; }
    if (e > 0 && e < 4 && slice_of(s, q)->slice_type == H264R_SLICE_P && q->mb_type == H264R_P_SKIP) { memset(St, 0, 16); return; }
    for (int x4 = 0; x4 < 4; ++x4) {
        int v;
        if (((q->cbp_blks >> ((lyq & 12) + x4)) & 1) || ((pm->cbp_blks >> ((lyp & 12) + x4)) & 1)) v = 2;
        else if (mixed) v = 1;
        else if (e > 0 && e < 4 && (q->mb_type == H264R_P_16x16 || q->mb_type == H264R_P_8x16)) v = 0;
        else {
            mvinfo_t mq = mvinfo(s, xq / 4 + x4, mbaff_mvinfo_row(s, Q, lyq));
            mvinfo_t mp = mvinfo(s, xq / 4 + x4, mbaff_mvinfo_row(s, P, lyp));
            v = bs_compare_mvs(&mq, &mp, mvlimit);
        }
        memset(St + 4 * x4, v, 4);
    }
}

static void strength_mbaff(pstate* s, int addr)                          /* deblock.cc:230-289 */
{
    const h264r_mb* q = mb_at(s, addr);
    const h264r_slice* sl = slice_of(s, q);
    memset(s->fver[addr], 0, sizeof(s->fver[addr]));
    memset(s->fhor[addr], 0, sizeof(s->fhor[addr]));
    memset(s->fhor4[addr], 0, sizeof(s->fhor4[addr]));
    if (sl->deblock_idc == 1) return;
    const int fq = is_field_mb(s, addr), dy = 1 + fq;
    int xq, yq;
    mbaff_loc(s, addr, 16, 16, 0, 0, &xq, &yq);
    const int L = mbaff_mb_at(s, 16, 16, xq - 1, yq, NULL), U = mbaff_mb_at(s, 16, 16, xq, yq - dy, NULL);
    int fl = 0, ft = 0;
    if (sl->deblock_idc == 0) { fl = L >= 0; ft = U >= 0; }
    else if (sl->deblock_idc == 2) {
        fl = L >= 0 && mb_at(s, L)->slice == q->slice;
        ft = U >= 0 && mb_at(s, U)->slice == q->slice;
    }
    for (int c = 0; c < 2; ++c) {
        s->fver[addr][c][0] = fl; s->fhor[addr][c][0] = ft;
        for (int e = 1; e < 4; ++e) s->fver[addr][c][e] = s->fhor[addr][c][e] = 1;
        s->fhor4[addr][c] = ft && !fq && is_field_mb(s, U);
    }
    if (q->flags & H264R_MBF_T8x8) s->fver[addr][0][1] = s->fver[addr][0][3] = s->fhor[addr][0][1] = s->fhor[addr][0][3] = 0;
    s->fver[addr][1][2] = s->fver[addr][1][3] = s->fhor[addr][1][2] = s->fhor[addr][1][3] = 0;
    for (int e = 0; e < 4; ++e) {
        if (s->fver[addr][0][e]) strength_vertical_mbaff(s, addr, e);
        if (s->fhor[addr][0][e]) strength_horizontal_mbaff(s, addr, e);
        if (e == 0 && s->fhor4[addr][0]) strength_horizontal_mbaff(s, addr, 4);
    }
}

/* filter_edge (deblock.cc:418-486) on an MBAFF frame: `edge` the sample offset, or 1 for the second
   field edge of a frame MB under a field pair (strength_hor[4], rows 1, 3, 5 against -1, -3, -5) */
static void filter_edge_mbaff(pstate* s, int addr, int chroma, int pl, int vertical, int fmode, int edge)
{
    const h264r_mb* q = mb_at(s, addr);
    const h264r_slice* sl = slice_of(s, q);
    const uint8_t* St = vertical ? s->strength_ver[addr][chroma ? edge * 4 / 8 : edge / 4]
                      : edge == 1 ? s->strength_hor4[addr] : s->strength_hor[addr][chroma ? edge * 4 / 8 : edge / 4];
    const int nE = chroma ? 8 : 16, pitch = chroma ? s->Wc : s->W, dy = 1 + fmode;
    int xI, yI;
    mbaff_loc(s, addr, 16, 16, 0, 0, &xI, &yI);
    const int xP = chroma ? xI / 2 : xI, yP = chroma ? (yI + 1) / 2 : yI;
    int xJ = xI, yJ = yI;
    if (vertical) xJ += (edge - 1) * (chroma ? 2 : 1);
    else yJ += dy * (edge - 1) * (chroma ? 2 : 1) - (edge % 2);
    int P = mbaff_mb_at(s, 16, 16, xJ, yJ, NULL);
    uint8_t* img = s->p->out[pl];
    const int incQ = vertical ? 1 : dy * pitch, nxtQ = vertical ? dy * pitch : 1;
    uint8_t* src = vertical ? &img[yP * pitch + xP + edge] : &img[(yP + dy * edge - (edge % 2)) * pitch + xP];
    const int mixed = vertical && !is_field_mb(s, addr) && is_field_mb(s, P);
    for (int pel = 0; pel < nE; ++pel, src += nxtQ) {
        const int bS = St[nE == 8 ? (pel << 1) + (mixed && (pel & 1)) : pel];
        if (!bS) continue;
        if (vertical) P = mbaff_mb_at(s, 16, 16, xJ, yI + dy * pel * (chroma ? 2 : 1) + (chroma && mixed && (pel & 1)), NULL);
        const h264r_mb* pm = mb_at(s, P);
        const int qPp = chroma ? pm->qp_c[pl - 1] : pm->qp_y, qPq = chroma ? q->qp_c[pl - 1] : q->qp_y;
        const int qPav = (qPp + qPq + 1) >> 1;
        const int indexA = clip3(0, 51, qPav + sl->filter_offset_a), indexB = clip3(0, 51, qPav + sl->filter_offset_b);
        filter_line(src, incQ, TABLE_ALPHA[indexA], TABLE_BETA[indexB], bS, chroma, bS < 4 ? TABLE_TC0[indexA][bS - 1] : 0);
    }
}

/* filter_vertical + filter_horizontal (deblock.cc:488-535) of one MB of an MBAFF frame */
static void filter_mb_mbaff(pstate* s, int a)
{
    const int fq = is_field_mb(s, a);
    for (int e = 0; e < 4; ++e) {
        if (s->fver[a][0][e]) filter_edge_mbaff(s, a, 0, 0, 1, fq, e * 4);
        if (s->fver[a][1][e]) { filter_edge_mbaff(s, a, 1, 1, 1, fq, e * 4); filter_edge_mbaff(s, a, 1, 2, 1, fq, e * 4); }
    }
    for (int e = 0; e < 4; ++e) {
        if (s->fhor[a][0][e]) {
            if (!(e == 0 && s->fhor4[a][0])) filter_edge_mbaff(s, a, 0, 0, 0, fq, e * 4);
            else { filter_edge_mbaff(s, a, 0, 0, 0, 1, 0); filter_edge_mbaff(s, a, 0, 0, 0, 1, 1); }
        }
        if (s->fhor[a][1][e]) {
            for (int pl = 1; pl <= 2; ++pl) {
                if (!(e == 0 && s->fhor4[a][1])) filter_edge_mbaff(s, a, 1, pl, 0, fq, e * 4);
                else { filter_edge_mbaff(s, a, 1, pl, 0, 1, 0); filter_edge_mbaff(s, a, 1, pl, 0, 1, 1); }
            }
        }
    }
}

/* MB address a of an MBAFF frame (pair a / 2, top or bottom) -> storage index */
static inline int mbaff_storage(const pstate* s, int a) { return ((a >> 1) / s->wmb * 2 + (a & 1)) * s->wmb + (a >> 1) % s->wmb; }

/* deblock_pic (deblock.cc:537-552) + the Deblock::deblock gate (:631-640). */
/* ---------------------------------------------------------------- 4:4:4 (ChromaArrayType 3)
 * Decoder::decode runs decode_one_component for PLANE_Y, PLANE_U and PLANE_V (decoder.cc:65-79):
 * each colour plane takes the LUMA prediction (intra_pred_* with the MB's luma modes, get_block_luma
 * with plane pl, inter_prediction.cc:158-340, its weights pred_weight_l[][pl][] and the chroma
 * denominator for pl > 0, :53-86), the luma residual path (coeff_luma_* / transform_luma_dc with
 * qp_scaled[pl] and plane pl's InvLevelScale, transform.cc:394-456, 825-854), and deblocking filters
 * it luma-style (chromaStyleFilteringFlag = chromaEdgeFlag && ChromaArrayType != 3, deblock.cc:422)
 * with the luma bS (strength_* read cbp_blks[0], :135,212; Strength index edge*4/MbWidthC) and QpC
 * of the plane (:469-470).  Planes never read each other, so a 4:4:4 picture is decoded here as
 * three pictures whose luma is plane pl, each through the 4:2:0 restatement above with plane
 * pl's QP, levels, weights, scaling lists and reference planes in the luma slots (their chroma
 * is scratch).  Pinned to the reference by its own 4:4:4 fixtures (tests/golden, ref_driver). */
static int derive_plane(const oracle_picture* p, int pl, oracle_picture* d, h264r_mb** mbs, h264r_slice** sl,
                        h264r_quant** q, uint8_t** scratch)
{
    const int n = p->width_mbs * p->height_mbs, ns = p->pic->num_slices;
    const size_t csz = (size_t)p->width_mbs * 8 * p->height_mbs * 8;
    *mbs = malloc(sizeof(h264r_mb) * (size_t)n);
    *sl = malloc(sizeof(h264r_slice) * (size_t)ns);
    *q = malloc(sizeof(h264r_quant));
    *scratch = malloc(2 * csz);
    if (!*mbs || !*sl || !*q || !*scratch) return H264R_ENOMEM;
    for (int a = 0; a < n; ++a) {
        h264r_mb m = p->mbs[a];
        const int cbpl = m.cbp & 15;
        if (m.mb_type == H264R_I_PCM) m.coef_off += 128u * (uint32_t)pl;           /* 256 samples per plane */
        else m.coef_off += (uint32_t)(pl * (64 * __builtin_popcount((unsigned)cbpl) + (m.mb_type == H264R_I_16x16 ? 16 : 0)));
        if (pl) { m.qp_y = m.qp_c[pl - 1]; m.qp_scaled[0] = m.qp_scaled[pl]; }
        m.cbp = (uint8_t)cbpl;
        m.chroma_mode = 0;
        (*mbs)[a] = m;
    }
    for (int i = 0; i < ns; ++i) {
        h264r_slice x = p->slices[i];
        if (pl) {
            for (int l = 0; l < 2; ++l)
                for (int r = 0; r < H264R_MAX_REFS; ++r) {
                    x.wp_weight[l][r][0] = x.wp_weight[l][r][pl];
                    x.wp_offset[l][r][0] = x.wp_offset[l][r][pl];
                }
            x.luma_log2_wd = x.chroma_log2_wd;
        }
        (*sl)[i] = x;
    }
    **q = *p->quant;
    for (int k = 0; k < 2; ++k) {
        memcpy((*q)->scale4x4[k][0], p->quant->scale4x4[k][pl], sizeof((*q)->scale4x4[k][0]));
        memcpy((*q)->scale8x8[k][0], p->quant->scale8x8[k][pl], sizeof((*q)->scale8x8[k][0]));
    }
    *d = *p;
    d->chroma_format = 1;
    d->mbs = *mbs; d->slices = *sl; d->quant = *q;
    for (int s = 0; s < H264R_MAX_SLOTS; ++s)
        for (int k = 0; k < 3; ++k) d->ref_planes[s][k] = p->ref_planes[s][pl];   /* chroma: scratch reads */
    d->out[0] = p->out[pl];
    d->out[1] = *scratch; d->out[2] = *scratch + csz;
    return 0;
}

/* 4:0:0 (ChromaArrayType 0): the luma of a 4:2:0 picture, no chroma at all (decoder.cc:199,
   deblock.cc:498,522 skip the chroma of ChromaArrayType 0) -- the first of decode_444's passes. */
static int decode_444(const oracle_picture* p, int what /* 1 reconstruct, 2 deblock, 3 both */)
{
    int st = 0;
    const int np = p->chroma_format == 0 ? 1 : 3;
    for (int pl = 0; pl < np && !st; ++pl) {
        oracle_picture d;
        h264r_mb* mbs = NULL; h264r_slice* sl = NULL; h264r_quant* q = NULL; uint8_t* scratch = NULL;
        st = derive_plane(p, pl, &d, &mbs, &sl, &q, &scratch);
        if (!st && (what & 1)) st = oracle_reconstruct_picture(&d);
        if (!st && (what & 2)) st = oracle_deblock_picture(&d);
        free(mbs); free(sl); free(q); free(scratch);
    }
    return st;
}

/* The picture geometry of a 4:2:0 or 4:2:2 picture (SubHeightC 2 / 1). */
static int init_state(pstate* s, const oracle_picture* p)
{
    memset(s, 0, sizeof(*s));
    s->p = p; s->wmb = p->width_mbs; s->hmb = p->height_mbs;
    s->cf = p->chroma_format == 2 ? 2 : 1;
    s->MHc = s->cf == 2 ? 16 : 8;
    s->W = s->wmb * 16; s->H = s->hmb * 16; s->Wc = s->wmb * 8; s->Hc = s->hmb * s->MHc; s->W4 = s->wmb * 4; s->H4 = s->hmb * 4;
    s->fld = p->pic->structure == H264R_TOP_FIELD || p->pic->structure == H264R_BOTTOM_FIELD;
    s->bot = p->pic->structure == H264R_BOTTOM_FIELD;
    s->mbaff = p->pic->structure == H264R_MBAFF_FRAME;
    if (s->mbaff && (s->hmb & 1)) return H264R_EINVAL;
    /* field pictures and MBAFF frames are on the 4:2:0 path only (the chroma field offset :348-361 is
       ChromaArrayType 1) */
    return (s->fld || s->mbaff) && s->cf != 1 ? H264R_EUNSUPPORTED : 0;
}

int oracle_deblock_picture(const oracle_picture* p)
{
    if (p->chroma_format == 3 || p->chroma_format == 0) return decode_444(p, 2);
    int n = p->width_mbs * p->height_mbs;
    pstate s;
    int st0 = init_state(&s, p);
    if (st0) return st0;
    int any = 0;
    for (int i = 0; i < p->pic->num_slices; ++i) any |= p->slices[i].deblock_idc != 1;
    if (!any) return 0;
    s.slice_nr = NULL;
    s.strength_ver = calloc((size_t)n, sizeof(*s.strength_ver));
    s.strength_hor = calloc((size_t)n, sizeof(*s.strength_hor));
    s.fver = calloc((size_t)n, sizeof(*s.fver));
    s.fhor = calloc((size_t)n, sizeof(*s.fhor));
    s.strength_hor4 = calloc((size_t)n, sizeof(*s.strength_hor4));
    s.fhor4 = calloc((size_t)n, sizeof(*s.fhor4));
    if (!s.strength_ver || !s.strength_hor || !s.fver || !s.fhor || !s.strength_hor4 || !s.fhor4) {
        free(s.strength_ver); free(s.strength_hor); free(s.fver); free(s.fhor); free(s.strength_hor4); free(s.fhor4);
        return H264R_ENOMEM;
    }
    if (s.mbaff) {                       /* MBAFF address order (deblock.cc:543-551) */
        for (int a = 0; a < n; ++a) strength_mbaff(&s, mbaff_storage(&s, a));
        for (int a = 0; a < n; ++a) filter_mb_mbaff(&s, mbaff_storage(&s, a));
        free(s.strength_ver); free(s.strength_hor); free(s.fver); free(s.fhor); free(s.strength_hor4); free(s.fhor4);
        return 0;
    }
    for (int a = 0; a < n; ++a) strength(&s, a);
    for (int a = 0; a < n; ++a) {
        /* filter_vertical (:488-504) then filter_horizontal (:506-535) */
        for (int e = 0; e < 4; ++e) {
            if (s.fver[a][0][e]) filter_edge(&s, a, 0, 0, 1, e * 4);
            if (s.fver[a][1][e]) { filter_edge(&s, a, 1, 1, 1, e * 4); filter_edge(&s, a, 1, 2, 1, e * 4); }
        }
        for (int e = 0; e < 4; ++e) {
            if (s.fhor[a][0][e]) filter_edge(&s, a, 0, 0, 0, e * 4);
            if (s.fhor[a][1][e]) { filter_edge(&s, a, 1, 1, 0, e * 4); filter_edge(&s, a, 1, 2, 0, e * 4); }
        }
    }
    free(s.strength_ver); free(s.strength_hor); free(s.fver); free(s.fhor); free(s.strength_hor4); free(s.fhor4);
    return 0;
}

int oracle_reconstruct_picture(const oracle_picture* p)
{
    if (p->chroma_format == 3 || p->chroma_format == 0) return decode_444(p, 1);
    int n = p->width_mbs * p->height_mbs;
    pstate s;
    int st0 = init_state(&s, p);
    if (st0) return st0;
    s.slice_nr = malloc(sizeof(int16_t) * (size_t)n);
    if (!s.slice_nr) return H264R_ENOMEM;
    for (int a = 0; a < n; ++a) s.slice_nr[a] = -1;
    int st = 0;
    for (int a = 0; a < n && !st; ++a) st = decode_mb(&s, s.mbaff ? mbaff_storage(&s, a) : a);
    free(s.slice_nr);
    return st;
}

int oracle_decode_picture(const oracle_picture* p)
{
    if (p->chroma_format == 3 || p->chroma_format == 0) return decode_444(p, 3);
    int st = oracle_reconstruct_picture(p);
    if (st) return st;
    return oracle_deblock_picture(p);
}

typedef struct { const oracle_picture* pics; int n, tid, threads, status; } job_t;
static void* worker(void* arg)
{
    job_t* j = (job_t*)arg;
    for (int i = j->tid; i < j->n; i += j->threads) {
        int st = oracle_decode_picture(&j->pics[i]);
        if (st) j->status = st;
    }
    return NULL;
}

int oracle_decode_pictures(const oracle_picture* pics, int n, int threads)
{
    if (threads <= 1) {
        for (int i = 0; i < n; ++i) { int st = oracle_decode_picture(&pics[i]); if (st) return st; }
        return 0;
    }
    pthread_t th[256];
    job_t jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; ++t) {
        jobs[t].pics = pics; jobs[t].n = n; jobs[t].tid = t; jobs[t].threads = threads; jobs[t].status = 0;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    int st = 0;
    for (int t = 0; t < threads; ++t) { pthread_join(th[t], NULL); if (jobs[t].status) st = jobs[t].status; }
    return st;
}
