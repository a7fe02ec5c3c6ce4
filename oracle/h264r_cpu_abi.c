/*
 * h264r_cpu_abi.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The per-picture streaming entry points of include/h264r.h implemented on the CPU
 * oracle (oracle/h264r_oracle.c), so that the reference's own parser + the drop-in
 * Decoder shim (shim/decoder_h264r.cc) can be linked and run in this container, which
 * has no GPU: oracle/_ref/ldecod_shim (oracle/Makefile `ref`).  It checks that the shim
 * feeds the boundary exactly what the reference reconstructs from (the shim build's
 * YUV == the unmodified reference's YUV), and it records what crossed the boundary:
 * with H264R_CAPTURE=<file> every picture's arrays (MB records, level pool, motion,
 * slices, picture parameters, quantisation tables, keep slot) and the oracle's planes
 * are appended to <file>, the replay fixtures of tests/test_stream_parity.py, which the
 * GPU tests decode through libh264r.so.  Never linked into the product.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "h264r.h"
#include "h264r_oracle.h"

struct h264r_ctx {
    int max_w, max_h;
    int cf, cb;                 /* chroma_format_idc and chroma bytes per MB and plane (64, 128, 256) */
    uint8_t* slot[H264R_MAX_SLOTS][3];
    int slot_w[H264R_MAX_SLOTS], slot_h[H264R_MAX_SLOTS];
    int in_pic, pw, ph;
    h264r_mb* mbs;
    uint8_t* seen;
    int16_t* levels;
    size_t n_levels, cap_levels;
    uint32_t* mv;
    int8_t* ref;
    h264r_slice* slices;
    h264r_pic pic;
    h264r_quant quant;
    uint8_t* async_out[2];      /* h264r_picture_end_async staging, Y | Cb | Cr */
    size_t async_n[2];
    int async_head, n_async;
};

static const int DQ4[6][3] = {{10, 13, 16}, {11, 14, 18}, {13, 16, 20}, {14, 18, 23}, {16, 20, 25}, {18, 23, 29}};
static const int DQ8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                              {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};

/* LevelScale(m, i, j): dequant_coef / dequant_coef8 of transform.cc:93-170 */
static int norm4(int m, int i, int j)
{
    if ((i & 1) == 0 && (j & 1) == 0) return DQ4[m][0];
    if ((i & 1) && (j & 1)) return DQ4[m][2];
    return DQ4[m][1];
}
static int norm8(int m, int i, int j)
{
    if (i % 4 == 0 && j % 4 == 0) return DQ8[m][0];
    if (i % 2 == 1 && j % 2 == 1) return DQ8[m][1];
    if (i % 4 == 2 && j % 4 == 2) return DQ8[m][2];
    if ((i % 4 == 0 && j % 2 == 1) || (i % 2 == 1 && j % 4 == 0)) return DQ8[m][3];
    if ((i % 4 == 0 && j % 4 == 2) || (i % 4 == 2 && j % 4 == 0)) return DQ8[m][4];
    return DQ8[m][5];
}

int h264r_abi_version(void) { return H264R_ABI_VERSION; }
const char* h264r_strerror(int s)
{
    switch (s) {
    case H264R_OK: return "ok";
    case H264R_EINVAL: return "invalid argument";
    case H264R_ENOMEM: return "out of memory";
    case H264R_ESTATE: return "call out of order";
    case H264R_EUNSUPPORTED: return "unsupported configuration";
    default: return "error";
    }
}
int h264r_device_count(void) { return 0; }

int h264r_quant_init_flat(h264r_quant* q)
{
    if (!q) return H264R_EINVAL;
    oracle_quant_init_flat(q);
    return H264R_OK;
}

int h264r_quant_init_lists(h264r_quant* q, const int32_t* const qm[12])
{
    if (!q || !qm) return H264R_EINVAL;
    for (int pl = 0; pl < 3; ++pl)
        for (int m = 0; m < 6; ++m) {
            for (int k = 0; k < 16; ++k) {
                q->scale4x4[0][pl][m][k] = (int16_t)(norm4(m, k / 4, k % 4) * qm[pl][k]);
                q->scale4x4[1][pl][m][k] = (int16_t)(norm4(m, k / 4, k % 4) * qm[3 + pl][k]);
            }
            for (int k = 0; k < 64; ++k) {
                q->scale8x8[0][pl][m][k] = (int16_t)(norm8(m, k / 8, k % 8) * qm[6 + 2 * pl][k]);
                q->scale8x8[1][pl][m][k] = (int16_t)(norm8(m, k / 8, k % 8) * qm[7 + 2 * pl][k]);
            }
        }
    return H264R_OK;
}

int h264r_create(h264r_ctx** out, int device, int max_w, int max_h, int chroma_format_idc, int bit_depth)
{
    (void)device;
    if (!out || max_w <= 0 || max_h <= 0) return H264R_EINVAL;
    if (chroma_format_idc < 0 || chroma_format_idc > 3 || bit_depth != 8) return H264R_EUNSUPPORTED;
    h264r_ctx* c = (h264r_ctx*)calloc(1, sizeof(h264r_ctx));
    if (!c) return H264R_ENOMEM;
    c->max_w = max_w; c->max_h = max_h;
    c->cf = chroma_format_idc;
    c->cb = chroma_format_idc == 3 ? 256 : chroma_format_idc == 2 ? 128 : chroma_format_idc == 1 ? 64 : 0;
    *out = c;
    return H264R_OK;
}

static void free_pic(h264r_ctx* c)
{
    free(c->mbs); free(c->seen); free(c->levels); free(c->mv); free(c->ref); free(c->slices);
    c->mbs = NULL; c->seen = NULL; c->levels = NULL; c->mv = NULL; c->ref = NULL; c->slices = NULL;
    c->n_levels = c->cap_levels = 0;
}

int h264r_destroy(h264r_ctx* c)
{
    if (!c) return H264R_EINVAL;
    for (int s = 0; s < H264R_MAX_SLOTS; ++s) free(c->slot[s][0]);
    free(c->async_out[0]);
    free(c->async_out[1]);
    free_pic(c);
    free(c);
    return H264R_OK;
}

static int ensure_slot(h264r_ctx* c, int s, int w, int h)
{
    if (c->slot[s][0] && c->slot_w[s] == w && c->slot_h[s] == h) return H264R_OK;
    free(c->slot[s][0]);
    size_t ys = (size_t)w * h * 256, cs = (size_t)w * h * c->cb;
    uint8_t* b = (uint8_t*)calloc(ys + 2 * cs, 1);
    if (!b) return H264R_ENOMEM;
    c->slot[s][0] = b; c->slot[s][1] = b + ys; c->slot[s][2] = b + ys + cs;
    c->slot_w[s] = w; c->slot_h[s] = h;
    return H264R_OK;
}

int h264r_set_ref(h264r_ctx* c, int slot, const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h)
{
    if (!c || slot < 0 || slot >= H264R_MAX_SLOTS || !y || (c->cb && (!u || !v))) return H264R_EINVAL;
    int st = ensure_slot(c, slot, w, h);
    if (st) return st;
    memcpy(c->slot[slot][0], y, (size_t)w * h * 256);
    if (c->cb) {
        memcpy(c->slot[slot][1], u, (size_t)w * h * c->cb);
        memcpy(c->slot[slot][2], v, (size_t)w * h * c->cb);
    }
    return H264R_OK;
}

int h264r_ref_planes(h264r_ctx* c, int slot, uint8_t** y, uint8_t** u, uint8_t** v)
{
    if (!c || slot < 0 || slot >= H264R_MAX_SLOTS) return H264R_EINVAL;
    if (y) *y = c->slot[slot][0];
    if (u) *u = c->slot[slot][1];
    if (v) *v = c->slot[slot][2];
    return c->slot[slot][0] ? H264R_OK : H264R_ESTATE;
}

int h264r_picture_begin(h264r_ctx* c, int w, int h, const h264r_pic* pic, const h264r_slice* slices,
                        const h264r_quant* quant)
{
    if (!c || !pic || !slices || !quant || w <= 0 || h <= 0 || w > c->max_w || h > c->max_h ||
        pic->num_slices <= 0 || pic->num_slices > H264R_MAX_SLICES)
        return H264R_EINVAL;
    free_pic(c);
    const size_t n = (size_t)w * h;
    c->pw = w; c->ph = h;
    c->mbs = (h264r_mb*)calloc(n, sizeof(h264r_mb));
    c->seen = (uint8_t*)calloc(n, 1);
    c->mv = (uint32_t*)calloc(2 * 16 * n, 4);
    c->ref = (int8_t*)malloc(2 * 16 * n);
    c->slices = (h264r_slice*)malloc(sizeof(h264r_slice) * pic->num_slices);
    if (!c->mbs || !c->seen || !c->mv || !c->ref || !c->slices) return H264R_ENOMEM;
    memset(c->ref, -1, 2 * 16 * n);
    memcpy(c->slices, slices, sizeof(h264r_slice) * pic->num_slices);
    c->pic = *pic;
    c->quant = *quant;
    c->in_pic = 1;
    return H264R_OK;
}

int h264r_mb_submit(h264r_ctx* c, int addr, const h264r_mb* mb, const int16_t* levels, int n_levels,
                    const uint32_t* mv, const int8_t* ref_idx)
{
    if (!c) return H264R_EINVAL;
    if (!c->in_pic) return H264R_ESTATE;
    const int n = c->pw * c->ph;
    if (addr < 0 || addr >= n || !mb || n_levels < 0 || (n_levels && !levels) || !mv || !ref_idx) return H264R_EINVAL;
    if (mb->slice >= c->pic.num_slices) return H264R_EINVAL;
    if (mb->mb_type == H264R_SI) return H264R_EUNSUPPORTED;
    size_t off = (c->n_levels + 7) & ~(size_t)7;
    if (off + (size_t)n_levels + 8 > c->cap_levels) {
        size_t cap = (off + n_levels + 8) * 2;
        int16_t* p = (int16_t*)realloc(c->levels, cap * 2);
        if (!p) return H264R_ENOMEM;
        memset(p + c->cap_levels, 0, (cap - c->cap_levels) * 2);
        c->levels = p; c->cap_levels = cap;
    }
    memcpy(c->levels + off, levels, (size_t)n_levels * 2);
    c->n_levels = off + n_levels;
    h264r_mb m = *mb;
    m.coef_off = (uint32_t)off;
    c->mbs[addr] = m;
    const int W4 = c->pw * 4, plane = W4 * c->ph * 4, x = addr % c->pw, y = addr / c->pw;
    for (int l = 0; l < 2; ++l)
        for (int k = 0; k < 16; ++k) {
            int idx = (y * 4 + k / 4) * W4 + x * 4 + k % 4;
            c->mv[(size_t)l * plane + idx] = mv[l * 16 + k];
            c->ref[(size_t)l * plane + idx] = ref_idx[l * 16 + k];
        }
    c->seen[addr] = 1;
    return H264R_OK;
}

/* Capture record (little-endian): int32 header[8] = {'H4RC', W, H, num_slices, n_levels,
 * keep_slot, chroma_format_idc, 1}, then mbs, levels, mv, ref_idx, slices, pic, quant, Y, Cb, Cr
 * (header[7] 1: header[6] holds the chroma format; 0 in captures older than that: 4:2:0). */
static void capture(const h264r_ctx* c, int keep, uint8_t* const out[3])
{
    const char* path = getenv("H264R_CAPTURE");
    if (!path) return;
    FILE* f = fopen(path, "ab");
    if (!f) return;
    const size_t n = (size_t)c->pw * c->ph;
    int32_t hdr[8] = {0x43523448, c->pw, c->ph, c->pic.num_slices, (int32_t)c->n_levels, keep, c->cf, 1};
    fwrite(hdr, 4, 8, f);
    fwrite(c->mbs, sizeof(h264r_mb), n, f);
    fwrite(c->levels, 2, c->n_levels, f);
    fwrite(c->mv, 4, 2 * 16 * n, f);
    fwrite(c->ref, 1, 2 * 16 * n, f);
    fwrite(c->slices, sizeof(h264r_slice), c->pic.num_slices, f);
    fwrite(&c->pic, sizeof(h264r_pic), 1, f);
    fwrite(&c->quant, sizeof(h264r_quant), 1, f);
    fwrite(out[0], 1, n * 256, f);
    fwrite(out[1], 1, n * c->cb, f);
    fwrite(out[2], 1, n * c->cb, f);
    fclose(f);
}

static int picture_end(h264r_ctx* c, uint8_t* y, uint8_t* u, uint8_t* v, int keep)
{
    if (!c->in_pic) return H264R_ESTATE;
    c->in_pic = 0;
    const int n = c->pw * c->ph;
    for (int a = 0; a < n; ++a) if (!c->seen[a]) return H264R_ESTATE;
    if (keep >= H264R_MAX_SLOTS || !y || (c->cb && (!u || !v))) return H264R_EINVAL;
    if (!c->levels) { c->levels = (int16_t*)calloc(8, 2); c->cap_levels = 8; }
    if (c->cf == 0 && c->cap_levels < c->n_levels + 64) {     /* the chroma view of a 4:0:0 PCM MB */
        int16_t* q = (int16_t*)realloc(c->levels, (c->n_levels + 64) * 2);
        if (!q) return H264R_ENOMEM;
        memset(q + c->cap_levels, 0, (c->n_levels + 64 - c->cap_levels) * 2);
        c->levels = q; c->cap_levels = c->n_levels + 64;
    }
    if (c->pic.structure < H264R_FRAME || c->pic.structure > H264R_MBAFF_FRAME) return H264R_EINVAL;
    /* a field picture's slots are frames of twice its height (include/h264r.h); an MBAFF frame is a frame */
    const int fld = c->pic.structure == H264R_TOP_FIELD || c->pic.structure == H264R_BOTTOM_FIELD, frame_h = c->ph << fld;
    oracle_picture p;
    memset(&p, 0, sizeof(p));
    p.width_mbs = c->pw; p.height_mbs = c->ph;
    p.mbs = c->mbs; p.levels = c->levels; p.mv = c->mv; p.ref_idx = c->ref;
    p.slices = c->slices; p.pic = &c->pic; p.quant = &c->quant;
    for (int s = 0; s < H264R_MAX_SLOTS; ++s)
        if (c->slot[s][0] && c->slot_w[s] == c->pw && c->slot_h[s] == frame_h)
            for (int k = 0; k < 3; ++k) p.ref_planes[s][k] = c->slot[s][k];
    p.out[0] = y; p.out[1] = u; p.out[2] = v;
    p.chroma_format = c->cf;
    if (fld && c->cf != 1) return H264R_EUNSUPPORTED;          /* field pictures: 4:2:0 only */
    int st = oracle_decode_picture(&p);
    if (st) {
        if (getenv("H264R_CPU_VERBOSE")) fprintf(stderr, "h264r (cpu): oracle_decode_picture -> %d\n", st);
        return H264R_EINVAL;
    }
    uint8_t* out[3] = {y, u, v};
    capture(c, keep, out);
    if (keep >= 0 && !fld) {
        if ((st = h264r_set_ref(c, keep, y, u, v, c->pw, c->ph))) return st;
    } else if (keep >= 0) {
        /* a field into its parity's rows of the slot's frame (dpb_combine_field_yuv
           picture.cc:578-622), the other field's rows left as they are */
        if ((st = ensure_slot(c, keep, c->pw, frame_h))) return st;
        const int bot = c->pic.structure == H264R_BOTTOM_FIELD;
        for (int k = 0; k < 3; ++k) {
            const int w = k ? c->pw * 8 : c->pw * 16, h = k ? c->ph * 8 : c->ph * 16;
            for (int r = 0; r < h; ++r) memcpy(c->slot[keep][k] + (size_t)(2 * r + bot) * w, out[k] + (size_t)r * w, w);
        }
    }
    return H264R_OK;
}

/* The asynchronous form: the CPU computes the picture at once into one of two staging sets,
 * h264r_picture_wait hands them out oldest first (the GPU library's contract). */
int h264r_picture_end_async(h264r_ctx* c, int keep)
{
    if (!c) return H264R_EINVAL;
    if (c->n_async == 2) return H264R_ESTATE;
    const size_t n = (size_t)c->pw * c->ph;
    const int k = (c->async_head + c->n_async) % 2;
    uint8_t* buf = (uint8_t*)realloc(c->async_out[k], n * (256 + 2 * c->cb));
    if (!buf) return H264R_ENOMEM;
    c->async_out[k] = buf;
    c->async_n[k] = n;
    int st = picture_end(c, buf, buf + n * 256, buf + n * (256 + c->cb), keep);
    if (st) return st;
    ++c->n_async;
    return H264R_OK;
}

int h264r_picture_wait(h264r_ctx* c, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!c) return H264R_EINVAL;
    if (!c->n_async) return H264R_ESTATE;
    const int k = c->async_head;
    const size_t n = c->async_n[k];
    const uint8_t* buf = c->async_out[k];
    if (y) memcpy(y, buf, n * 256);
    if (u) memcpy(u, buf + n * 256, n * c->cb);
    if (v) memcpy(v, buf + n * (256 + c->cb), n * c->cb);
    c->async_head = (k + 1) % 2;
    --c->n_async;
    return H264R_OK;
}

int h264r_picture_end(h264r_ctx* c, uint8_t* y, uint8_t* u, uint8_t* v, int keep)
{
    if (!c) return H264R_EINVAL;
    if (c->n_async) return H264R_ESTATE;
    return picture_end(c, y, u, v, keep);
}

int h264r_check(h264r_ctx* c) { return c ? H264R_OK : H264R_EINVAL; }
