/*
 * synth.c -- seeded synthetic post-entropy workload (include/h264r_synth.h).
 *
 * Distributions follow SURVEY.md section 8(d).  Everything the reference
 * decoder would assert on is avoided by construction: intra prediction modes
 * are drawn from the modes whose neighbours are available under the
 * reference's availability rules (intra_prediction.cc:137-187, 359-411,
 * 624-666, 748-796), unused motion lists carry ref_idx -1 and a zero MV
 * (interpret_mb.cc:583-591), I_16x16 AC and chroma AC blocks never carry a
 * level at scan position 0, and cbp_blks is derived from the levels exactly as
 * coeff_luma_ac does (transform.cc:431-436; 0xFFFF for I_PCM, interpret_mb.cc:421).
 */
#include "h264r_synth.h"

#include <string.h>

/* ------------------------------------------------------------------ PRNG */
typedef struct { uint64_t s; } rng_t;
static uint64_t next64(rng_t* r)
{
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static int rnd(rng_t* r, int n) { return (int)(next64(r) % (uint64_t)n); }        /* [0, n) */
static int rrange(rng_t* r, int lo, int hi) { return lo + rnd(r, hi - lo + 1); }   /* [lo, hi] */

static const uint8_t QP_SCALE_CR[52] = {                  /* interpret_mb.cc:777-782 */
    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
    26, 27, 28, 29, 29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

static int clip3i(int lo, int hi, int x) { return x < lo ? lo : (x > hi ? hi : x); }

int h264r_synth_slot_poc(int slot) { return 4 * slot; }
/* a field picture (PAFF); an MBAFF frame is a frame picture for its lists and POCs */
static int field_pic(const h264r_synth_cfg* c)
{
    return c->structure == H264R_TOP_FIELD || c->structure == H264R_BOTTOM_FIELD;
}
int h264r_synth_ref_frames(const h264r_synth_cfg* cfg)
{
    return field_pic(cfg) ? (cfg->num_refs + 1) / 2 : cfg->num_refs;
}
int h264r_synth_cur_poc(const h264r_synth_cfg* cfg)
{
    /* P: after every reference; B: between slot (n/2 - 1) and slot n/2 (n DPB frames); a
       bottom field one after its top field */
    const int n = h264r_synth_ref_frames(cfg), bot = cfg->structure == H264R_BOTTOM_FIELD;
    if (cfg->kind == H264R_SYNTH_B && n >= 2) return 4 * (n / 2) - 2 + bot;
    return 4 * n + bot;
}

/* POC of list candidate k: frame slot k (frames), or field k of the DPB frames (slot k / 2,
   bottom when k is odd) */
static int cand_poc(const h264r_synth_cfg* c, int k)
{
    return field_pic(c) ? h264r_synth_slot_poc(k >> 1) + (k & 1) : h264r_synth_slot_poc(k);
}
static int cand_ref(const h264r_synth_cfg* c, int k)
{
    return field_pic(c) ? (k >> 1) | ((k & 1) ? H264R_REF_BOTTOM : 0) : k;
}
static int ref_poc(int ref) { return h264r_synth_slot_poc(ref & 31) + ((ref & H264R_REF_BOTTOM) ? 1 : 0); }

int h264r_synth_default(h264r_synth_cfg* c, int config_idx, int width_mbs, int height_mbs)
{
    memset(c, 0, sizeof(*c));
    c->width_mbs = width_mbs; c->height_mbs = height_mbs;
    c->num_slices = 1; c->deblock_idc = 0; c->num_refs = 2;
    c->qp_min = 20; c->qp_max = 40; c->intra_permille = 100;
    c->mv_range_x = 64; c->mv_range_y = 32;
    c->seed = 0x2640ull + (uint64_t)config_idx;
    switch (config_idx) {
    case 1: case 2: c->kind = H264R_SYNTH_INTRA; c->transform8x8 = 1; c->num_refs = 0; break;
    case 3: c->kind = H264R_SYNTH_P; break;
    case 4: c->kind = H264R_SYNTH_B; c->transform8x8 = 1; c->num_slices = 4; c->deblock_idc = 2; c->wp_mode = 2; break;
    case 5: c->kind = H264R_SYNTH_B; c->transform8x8 = 1; c->num_slices = 8; c->deblock_idc = 2; c->wp_mode = 2; break;
    default: return H264R_EINVAL;
    }
    if (c->num_slices > height_mbs) c->num_slices = height_mbs;
    return H264R_OK;
}

/* ------------------------------------------------------------ slices */
static int slice_first_row(int s, int nslices, int hmb) { return (int)(((int64_t)s * hmb) / nslices); }
static int slice_of_row(int row, int nslices, int hmb)
{
    int s = 0;
    while (s + 1 < nslices && slice_first_row(s + 1, nslices, hmb) <= row) ++s;
    return s;
}

static void make_slices(const h264r_synth_cfg* c, rng_t* r, h264r_slice* sl)
{
    int cur = h264r_synth_cur_poc(c);
    int n = c->num_refs;
    for (int s = 0; s < c->num_slices; ++s) {
        h264r_slice* x = &sl[s];
        memset(x, 0, sizeof(*x));
        x->slice_type = c->kind == H264R_SYNTH_INTRA ? H264R_SLICE_I : c->kind == H264R_SYNTH_P ? H264R_SLICE_P : H264R_SLICE_B;
        x->deblock_idc = (uint8_t)c->deblock_idc;
        x->filter_offset_a = (int8_t)c->filter_offset_a;
        x->filter_offset_b = (int8_t)c->filter_offset_b;
        x->wp_mode = (uint8_t)c->wp_mode;
        x->luma_log2_wd = 5; x->chroma_log2_wd = 5;
        if (c->kind == H264R_SYNTH_INTRA) continue;
        if (c->kind == H264R_SYNTH_P && c->sp_slices) {
            x->slice_type = H264R_SLICE_SP;
            x->qs_y = (uint8_t)rrange(r, 0, 5);
            x->sp_switch = (uint8_t)rrange(r, 0, 1);
            x->qs_c[0] = x->qs_c[1] = (int8_t)x->qs_y;     /* chroma_qp_index_offset 0, QsY < 30 */
        }
        /* L0: descending POC below cur then ascending above; L1: the reverse (8.2.4.2.3 style;
           fields: the candidates are the DPB frames' fields, so the order alternates parity) */
        int l0[2 * H264R_MAX_REFS], l1[2 * H264R_MAX_REFS], k0 = 0, k1 = 0;
        const int nc = field_pic(c) ? 2 * h264r_synth_ref_frames(c) : n;
        for (int k = nc - 1; k >= 0; --k) if (cand_poc(c, k) < cur) l0[k0++] = cand_ref(c, k);
        for (int k = 0; k < nc; ++k) if (cand_poc(c, k) > cur) l0[k0++] = cand_ref(c, k);
        for (int k = 0; k < nc; ++k) if (cand_poc(c, k) > cur) l1[k1++] = cand_ref(c, k);
        for (int k = nc - 1; k >= 0; --k) if (cand_poc(c, k) < cur) l1[k1++] = cand_ref(c, k);
        x->num_ref[0] = (uint8_t)n;
        x->num_ref[1] = (uint8_t)(c->kind == H264R_SYNTH_B ? n : 0);
        for (int i = 0; i < H264R_MAX_REFS; ++i) { x->ref_slot[0][i] = -1; x->ref_slot[1][i] = -1; }
        for (int i = 0; i < n; ++i) {
            x->ref_slot[0][i] = (int8_t)l0[i];
            if (c->kind == H264R_SYNTH_B) x->ref_slot[1][i] = (int8_t)l1[i];
        }
        if (c->wp_mode == 1) {        /* explicit: pred_weight_table (interpret_rbsp.cc:837-900) */
            x->luma_log2_wd = (uint8_t)rrange(r, 0, 7);
            x->chroma_log2_wd = (uint8_t)rrange(r, 0, 7);
            for (int l = 0; l < 2; ++l)
                for (int i = 0; i < n; ++i)
                    for (int pl = 0; pl < 3; ++pl) {
                        int d = pl ? x->chroma_log2_wd : x->luma_log2_wd;
                        int w = (1 << d) + rrange(r, -(1 << d) / 2 - 1, (1 << d) / 2 + 1);
                        x->wp_weight[l][i][pl] = (int8_t)clip3i(-128, 127, w);
                        x->wp_offset[l][i][pl] = (int8_t)rrange(r, -20, 20);
                    }
        } else if (c->wp_mode == 2) { /* implicit: inter_prediction.cc:112-139 */
            for (int i0 = 0; i0 < n; ++i0)
                for (int i1 = 0; i1 < n; ++i1) {
                    int p0 = ref_poc(x->ref_slot[0][i0]);
                    int p1 = ref_poc(x->ref_slot[1][i1] >= 0 ? x->ref_slot[1][i1] : 0);
                    int td = clip3i(-128, 127, p1 - p0), w1;
                    if (td == 0) w1 = 32;
                    else {
                        int tb = clip3i(-128, 127, cur - p0);
                        int tx = (16384 + (td / 2 < 0 ? -(td / 2) : td / 2)) / td;
                        int dsf = clip3i(-1024, 1023, (tx * tb + 32) >> 6);
                        w1 = dsf >> 2;
                        if (w1 < -64 || w1 > 128) w1 = 32;
                    }
                    x->implicit_w1[i0][i1] = (int16_t)w1;
                }
        }
    }
}

/* ------------------------------------------------------------ levels */
static int16_t gen_level(rng_t* r)
{
    if (rnd(r, 100) < 70) return 0;
    int mag = 1;
    while (mag < 8 && rnd(r, 2)) ++mag;            /* geometric on 1..8 */
    return (int16_t)(rnd(r, 2) ? mag : -mag);
}

/* ------------------------------------------------------------ picture */
typedef struct {
    const h264r_synth_cfg* c;
    int W4;
    h264r_mb* mbs;
    uint32_t* mv;
    int8_t* ref;
} gen_t;

/* ---- MBAFF frames: availability where Neighbour::get_neighbour finds a sample (neighbour.cc:
   123-173) -- the geometric frame sample at (xN, yN) of MB a's own sample grid (a field MB's rows
   are every second frame row of its pair), in the MB that holds it, decoded before a (MBAFF
   address order) and in a's slice (intra_prediction.cc:145-152).  maxW / maxH: 16 / 16 luma,
   8 / 8 chroma (4:2:0).  Returns the MB's storage index or -1. */
static int mbaff_nb(const gen_t* g, int a, int xN, int yN, int maxW, int maxH)
{
    const int W = g->c->width_mbs, HP = g->c->height_mbs / 2;
    const int mbx = a % W, mby = a / W, py = mby >> 1, b = mby & 1;
    const int fld = (g->mbs[a].flags & H264R_MBF_FIELD) != 0;
    const int gx = mbx * maxW + xN;
    const int gy = py * 2 * maxH + (fld ? b + 2 * yN : b * maxH + yN);
    if (gx < 0 || gx >= W * maxW || gy < 0 || gy >= HP * 2 * maxH) return -1;
    const int nx = gx / maxW, npy = gy / (2 * maxH);
    if (npy * W + nx > py * W + mbx) return -1;                 /* a later pair: not decoded */
    const int top = (2 * npy) * W + nx;
    const int nfld = (g->mbs[top].flags & H264R_MBF_FIELD) != 0;
    const int nb = nfld ? (gy & 1) : ((gy % (2 * maxH)) >= maxH);
    const int n = top + nb * W;
    if (n == a) return n;                                       /* inside the MB itself */
    if (npy * W + nx == py * W + mbx && nb >= b) return -1;     /* the pair's later MB */
    return g->mbs[n].slice == g->mbs[a].slice ? n : -1;
}
static int mbaff_intra_ok(const gen_t* g, int n)
{
    return n >= 0 && (!g->c->constrained_intra || (g->mbs[n].flags & H264R_MBF_INTRA));
}
/* left neighbours of rows y0 .. y0 + n - 1 at column x: available as the reference's ctor decides
   (non-CIP: the first row's MB; CIP: every row's MB intra, intra_prediction.cc:156-167) */
static int mbaff_left(const gen_t* g, int a, int x, int y0, int n, int maxW, int maxH)
{
    if (!g->c->constrained_intra) return mbaff_nb(g, a, x, y0, maxW, maxH) >= 0;
    for (int i = 0; i < n; ++i) if (!mbaff_intra_ok(g, mbaff_nb(g, a, x, y0 + i, maxW, maxH))) return 0;
    return 1;
}

static int mb_exists_same_slice(const gen_t* g, int addr, int nx, int ny)
{
    const h264r_synth_cfg* c = g->c;
    if (nx < 0 || ny < 0 || nx >= c->width_mbs || ny >= c->height_mbs) return 0;
    int n = ny * c->width_mbs + nx;
    if (n >= addr) return 0;   /* not decoded yet */
    return g->mbs[n].slice == g->mbs[addr].slice;
}

/* MB-level availability A,B,C,D for intra under constrained_intra_pred. */
static void mb_avail(const gen_t* g, int addr, int av[4])
{
    int x = addr % g->c->width_mbs, y = addr / g->c->width_mbs;
    int nx[4] = {x - 1, x, x + 1, x - 1}, ny[4] = {y, y - 1, y - 1, y - 1};
    for (int k = 0; k < 4; ++k) {
        av[k] = mb_exists_same_slice(g, addr, nx[k], ny[k]);
        if (av[k] && g->c->constrained_intra)
            av[k] = (g->mbs[ny[k] * g->c->width_mbs + nx[k]].flags & H264R_MBF_INTRA) != 0;
    }
}

static int pick_mode(rng_t* r, const int* modes, int n) { return modes[rnd(r, n)]; }

/* valid NxN modes given block-level availability of A (left), B (top), D (top-left) */
static int pick_nxn_mode(rng_t* r, int A, int B, int D)
{
    int m[9], k = 0;
    m[k++] = 2;
    if (B) { m[k++] = 0; m[k++] = 3; m[k++] = 7; }
    if (A) { m[k++] = 1; m[k++] = 8; }
    if (A && B && D) { m[k++] = 4; m[k++] = 5; m[k++] = 6; }
    return pick_mode(r, m, k);
}

static void set_motion(gen_t* g, int addr, int bx, int by, int bw, int bh, int r0, int r1,
                       uint32_t m0, uint32_t m1)
{
    int x = addr % g->c->width_mbs, y = addr / g->c->width_mbs;
    int plane = g->W4 * g->c->height_mbs * 4;
    for (int j = by; j < by + bh; ++j)
        for (int i = bx; i < bx + bw; ++i) {
            int idx = (y * 4 + j) * g->W4 + x * 4 + i;
            g->ref[idx] = (int8_t)r0; g->ref[plane + idx] = (int8_t)r1;
            g->mv[idx] = r0 >= 0 ? m0 : 0; g->mv[plane + idx] = r1 >= 0 ? m1 : 0;
        }
}

static uint32_t rand_mv(rng_t* r, const h264r_synth_cfg* c)
{
    int mx = rrange(r, -c->mv_range_x, c->mv_range_x) * 4 + rnd(r, 4);
    int my = rrange(r, -c->mv_range_y, c->mv_range_y) * 4 + rnd(r, 4);
    return (uint32_t)(uint16_t)(int16_t)mx | ((uint32_t)(uint16_t)(int16_t)my << 16);
}

/* One partition's motion: dir 0 L0, 1 L1, 2 Bi; dir < 0 draws it (B) or uses L0 (P). */
static void rand_partition_dir(gen_t* g, rng_t* r, int addr, int bx, int by, int bw, int bh, int bslice, int dir)
{
    int nref = g->c->num_refs;
    if (g->mbs[addr].flags & H264R_MBF_FIELD) nref *= 2;          /* MBAFF field MB: refIdx counts fields */
    if (dir < 0) dir = bslice ? rnd(r, 3) : 0;
    int r0 = (dir == 0 || dir == 2) ? rnd(r, nref) : -1;
    int r1 = (dir == 1 || dir == 2) ? rnd(r, nref) : -1;
    set_motion(g, addr, bx, by, bw, bh, r0, r1, rand_mv(r, g->c), rand_mv(r, g->c));
}
static void rand_partition(gen_t* g, rng_t* r, int addr, int bx, int by, int bw, int bh, int bslice)
{
    rand_partition_dir(g, r, addr, bx, by, bw, bh, bslice, -1);
}

int h264r_synth_picture(const h264r_synth_cfg* c, int index, h264r_mb* mbs, int16_t* levels,
                        int64_t* n_levels, uint32_t* mv, int8_t* ref_idx, h264r_slice* slices,
                        h264r_pic* pic)
{
    if (!c || !mbs || !levels || !mv || !ref_idx || !slices || !pic) return H264R_EINVAL;
    if (c->width_mbs <= 0 || c->height_mbs <= 0 || c->num_slices <= 0 || c->num_slices > H264R_MAX_SLICES ||
        c->num_slices > c->height_mbs || c->num_refs < 0 || c->num_refs > H264R_MAX_REFS ||
        c->structure < H264R_FRAME || c->structure > H264R_MBAFF_FRAME ||
        (c->structure == H264R_MBAFF_FRAME && ((c->height_mbs & 1) || c->num_slices > c->height_mbs / 2 ||
                                               (c->chroma_format != 0 && c->chroma_format != 1) || c->wp_mode == 2 ||
                                               c->sp_slices || c->lossless_permille)) ||
        (c->kind != H264R_SYNTH_INTRA && c->num_refs < 1) || c->qp_min < 0 || c->qp_max > 51 ||
        c->qp_min > c->qp_max || (c->chroma_format >= 2 && c->structure != H264R_FRAME) ||
        c->chroma_format < 0 || c->chroma_format > 4)
        return H264R_EINVAL;
    const int f444 = c->chroma_format == 3, f422 = c->chroma_format == 2,
              f400 = c->chroma_format == H264R_SYNTH_CHROMA_400;
    rng_t r = {c->seed * 0x100000001B3ull + (uint64_t)index * 0x9E3779B97F4A7C15ull + 1};
    int W = c->width_mbs, H = c->height_mbs, nmb = W * H;
    gen_t g = {c, W * 4, mbs, mv, ref_idx};
    memset(mbs, 0, sizeof(h264r_mb) * (size_t)nmb);
    memset(mv, 0, sizeof(uint32_t) * 2 * 16 * (size_t)nmb);
    memset(ref_idx, -1, 2 * 16 * (size_t)nmb);
    make_slices(c, &r, slices);
    pic->constrained_intra_pred = c->constrained_intra;
    pic->num_slices = c->num_slices;
    pic->poc = h264r_synth_cur_poc(c);
    pic->structure = c->structure;

    int64_t off = 0;
    int bslice = c->kind == H264R_SYNTH_B;
    const int mbaff = c->structure == H264R_MBAFF_FRAME;
    for (int k = 0; k < nmb; ++k) {
        /* MBAFF: MB address order, pair by pair (top, bottom), a = the storage index */
        const int a = mbaff ? ((k >> 1) / W * 2 + (k & 1)) * W + (k >> 1) % W : k;
        h264r_mb* m = &mbs[a];
        int mby = a / W;
        m->slice = (uint16_t)(mbaff ? slice_of_row(mby >> 1, c->num_slices, H / 2) : slice_of_row(mby, c->num_slices, H));
        if (mbaff) {
            /* mb_field_decoding_flag, one per pair (drawn with the top MB) */
            const int fld = (k & 1) ? (mbs[a - W].flags & H264R_MBF_FIELD) != 0 : rnd(&r, 2);
            m->flags = fld ? H264R_MBF_FIELD : 0;
        }
        const uint8_t fflag = m->flags;
        int is_intra;
        if (c->kind == H264R_SYNTH_INTRA) is_intra = 1;
        else is_intra = rnd(&r, 1000) < c->intra_permille;
        int pcm = is_intra && rnd(&r, 1000) < c->pcm_permille;

        int qp = rrange(&r, c->qp_min, c->qp_max);
        if (pcm) qp = 0;
        else if (c->lossless_permille && rnd(&r, 1000) < c->lossless_permille) qp = 0;
        /* TransformBypassModeFlag = qpprime_y_zero_transform_bypass_flag && qp_scaled[0] == 0
           (interpret_mb.cc:804); I_PCM ignores it */
        const int bypass = c->lossless_permille > 0 && qp == 0 && !pcm;
        m->qp_y = (int8_t)qp;
        int qc = clip3i(0, 51, qp);   /* chroma_qp_index_offset 0 (update_qp :784-805) */
        qc = qc < 30 ? qc : QP_SCALE_CR[qc];
        m->qp_c[0] = m->qp_c[1] = (int8_t)qc;
        m->qp_scaled[0] = (uint8_t)qp; m->qp_scaled[1] = m->qp_scaled[2] = (uint8_t)qc;
        m->coef_off = (uint32_t)off;

        if (pcm) {
            m->mb_type = H264R_I_PCM;
            m->flags = H264R_MBF_INTRA | fflag;
            m->cbp_blks = 0xFFFF;
            uint8_t* raw = (uint8_t*)(levels + off);
            const int npcm = f444 ? 768 : f422 ? 512 : f400 ? 256 : 384;   /* Y 256, Cb / Cr 64, 128 (4:2:2), 256 (4:4:4) */
            for (int k = 0; k < npcm; ++k) raw[k] = (uint8_t)rnd(&r, 256);
            off += npcm / 2;
            continue;
        }
        int cbpl = 0, cbpc = 0, t8 = 0;
        if (is_intra) {
            m->flags = H264R_MBF_INTRA | fflag;
            int kind = rnd(&r, 100);
            if (kind < 40) m->mb_type = H264R_I_4x4;
            else if (kind < 80) m->mb_type = c->transform8x8 ? H264R_I_8x8 : H264R_I_4x4;
            else m->mb_type = H264R_I_16x16;
            int av[4];
            if (mbaff) {
                av[0] = mbaff_left(&g, a, -1, 0, 16, 16, 16);
                av[1] = mbaff_intra_ok(&g, mbaff_nb(&g, a, 0, -1, 16, 16));
                av[2] = 0;
                av[3] = mbaff_intra_ok(&g, mbaff_nb(&g, a, -1, -1, 16, 16));
            } else
                mb_avail(&g, a, av);
            if (m->mb_type == H264R_I_16x16) {
                int md[4], k = 0;
                md[k++] = 2;
                if (av[1]) md[k++] = 0;
                if (av[0]) md[k++] = 1;
                if (av[0] && av[1] && av[3]) md[k++] = 3;
                m->i16_mode = (uint8_t)pick_mode(&r, md, k);
                cbpl = rnd(&r, 2) ? 15 : 0;
            } else {
                int size = m->mb_type == H264R_I_4x4 ? 4 : 8;
                t8 = size == 8;
                int nb = size == 4 ? 16 : 4;
                for (int b = 0; b < nb; ++b) {
                    int xO, yO;
                    if (size == 4) { xO = ((b / 4) % 2) * 8 + ((b % 4) % 2) * 4; yO = ((b / 4) / 2) * 8 + ((b % 4) / 2) * 4; }
                    else { xO = (b % 2) * 8; yO = (b / 2) * 8; }
                    int A = xO > 0 ? 1 : av[0];
                    int B = yO > 0 ? 1 : av[1];
                    int D = (xO > 0 && yO > 0) ? 1 : (xO == 0 && yO == 0) ? av[3] : (xO == 0 ? av[0] : av[1]);
                    if (mbaff) {         /* the block's own neighbours (intra_prediction.cc:137-187, 359-411) */
                        A = mbaff_left(&g, a, xO - 1, yO, size, 16, 16);
                        B = mbaff_intra_ok(&g, mbaff_nb(&g, a, xO, yO - 1, 16, 16));
                        D = mbaff_intra_ok(&g, mbaff_nb(&g, a, xO - 1, yO - 1, 16, 16));
                    }
                    int mode = pick_nxn_mode(&r, A, B, D);
                    m->ipred[b >> 1] |= (uint8_t)(mode << ((b & 1) * 4));
                }
                cbpl = rnd(&r, 16);
            }
            {
                int ca[4] = {av[0], av[1], av[0], av[3]};
                if (mbaff) {     /* chroma neighbours on the 8 x 8 grid (intra_prediction.cc:745-790) */
                    ca[0] = mbaff_left(&g, a, -1, 0, 4, 8, 8);
                    ca[2] = mbaff_left(&g, a, -1, 4, 4, 8, 8) && mbaff_nb(&g, a, -1, 0, 8, 8) >= 0;
                    ca[1] = mbaff_intra_ok(&g, mbaff_nb(&g, a, 0, -1, 8, 8));
                    ca[3] = mbaff_intra_ok(&g, mbaff_nb(&g, a, -1, -1, 8, 8));
                }
                int md[4], k = 0;
                md[k++] = 0;
                if (ca[0] && ca[2]) md[k++] = 1;
                if (ca[1]) md[k++] = 2;
                if (ca[0] && ca[2] && ca[1] && ca[3]) md[k++] = 3;
                m->chroma_mode = (uint8_t)pick_mode(&r, md, k);
            }
            cbpc = f444 || f400 ? 0 : rnd(&r, 3);
            if (f444 || f400) m->chroma_mode = 0;         /* no chroma intra mode in 4:4:4 / 4:0:0 */
        } else {
            int k = rnd(&r, 90);    /* conditional on inter: skip/16x16/16x8/8x16/8x8 = 15/45/10/10/10 */
            int mt = k < 15 ? H264R_P_SKIP : k < 60 ? H264R_P_16x16 : k < 70 ? H264R_P_16x8 : k < 80 ? H264R_P_8x16 : H264R_P_8x8;
            m->flags = fflag;
            m->mb_type = (uint8_t)mt;
            switch (mt) {
            case H264R_P_SKIP:
                if (!bslice) rand_partition(&g, &r, a, 0, 0, 4, 4, 0);
                else for (int b8 = 0; b8 < 4; ++b8) rand_partition(&g, &r, a, (b8 & 1) * 2, (b8 >> 1) * 2, 2, 2, 1);
                break;
            case H264R_P_16x16: rand_partition(&g, &r, a, 0, 0, 4, 4, bslice); break;
            case H264R_P_16x8: rand_partition(&g, &r, a, 0, 0, 4, 2, bslice); rand_partition(&g, &r, a, 0, 2, 4, 2, bslice); break;
            case H264R_P_8x16: rand_partition(&g, &r, a, 0, 0, 2, 4, bslice); rand_partition(&g, &r, a, 2, 0, 2, 4, bslice); break;
            default: {
                int all8x8 = 1;
                for (int b8 = 0; b8 < 4; ++b8) {
                    int bx = (b8 & 1) * 2, by = (b8 >> 1) * 2;
                    int st = rnd(&r, 4);   /* sub-type 8x8 / 8x4 / 4x8 / 4x4 */
                    int d8 = bslice ? rnd(&r, 3) : 0;   /* one pred dir per sub-MB (sub_mb_type, 7.4.5.2) */
                    if (st) all8x8 = 0;
                    if (st == 0) rand_partition_dir(&g, &r, a, bx, by, 2, 2, bslice, d8);
                    else if (st == 1) { rand_partition_dir(&g, &r, a, bx, by, 2, 1, bslice, d8); rand_partition_dir(&g, &r, a, bx, by + 1, 2, 1, bslice, d8); }
                    else if (st == 2) { rand_partition_dir(&g, &r, a, bx, by, 1, 2, bslice, d8); rand_partition_dir(&g, &r, a, bx + 1, by, 1, 2, bslice, d8); }
                    else for (int q = 0; q < 4; ++q) rand_partition_dir(&g, &r, a, bx + (q & 1), by + (q >> 1), 1, 1, bslice, d8);
                }
                /* transform_size_8x8 only without sub-8x8 partitions (7.3.5) */
                if (!all8x8) t8 = -1;
                break; }
            }
            int skip_res = mt == H264R_P_SKIP && (!bslice || rnd(&r, 2));
            if (!skip_res) { cbpl = rnd(&r, 16); cbpc = f444 || f400 ? 0 : rnd(&r, 3); }
            if (t8 == -1) t8 = 0;
            else t8 = c->transform8x8 && cbpl && rnd(&r, 2);
            if (mt == H264R_P_SKIP && !bslice) t8 = 0;
        }
        if (t8) m->flags |= H264R_MBF_T8x8;
        if (bypass) {
            m->flags |= H264R_MBF_BYPASS;
            /* an inter MB's Intra4x4PredMode / Intra8x8PredMode are whatever the mb_t slot
               held (macroblock_t::init, slice_data.cc:455-503, does not reset them), and the
               reference's bypass reads them for the DPCM direction (transform.cc:993,1008) */
            if (!is_intra)
                for (int b = 0; b < 8; ++b) m->ipred[b] = (uint8_t)(rnd(&r, 9) | (rnd(&r, 9) << 4));
        }
        m->cbp = (uint8_t)(cbpl | (cbpc << 4));

        /* levels, in the compacted layout of include/h264r.h */
        int i16 = m->mb_type == H264R_I_16x16;
        uint16_t blks = 0;
        for (int b8 = 0; b8 < 4; ++b8) {
            if (!(cbpl & (1 << b8))) continue;
            int16_t* blk = levels + off;
            int any8 = 0;
            for (int b4 = 0; b4 < 4; ++b4) {
                int any = 0;
                for (int pos = 0; pos < 16; ++pos) {
                    int16_t v = (i16 && pos == 0 && !t8) ? 0 : gen_level(&r);
                    blk[b4 * 16 + pos] = v;
                    any |= v != 0;
                }
                int bx = (b8 & 1) * 2 + (b4 & 1), by = (b8 >> 1) * 2 + (b4 >> 1);
                if (any && !t8) blks |= (uint16_t)(1u << (by * 4 + bx));
                any8 |= any;
            }
            if (any8 && t8) blks |= (uint16_t)(0x33u << (((b8 >> 1) * 2) * 4 + (b8 & 1) * 2));
            off += 64;
        }
        if (f422 || f400) {
            /* 4:2:2 (include/h264r.h): the I_16x16 DC right after the luma blocks, then chroma AC
               (2 planes x 8 blocks x 16) and chroma DC (2 x 8, raster of the 2x4 matrix) */
            if (i16) {
                for (int k = 0; k < 16; ++k) levels[off + k] = gen_level(&r);
                off += 16;
            }
            if (cbpc == 2) {
                for (int k = 0; k < 256; ++k) levels[off + k] = (k % 16 == 0) ? 0 : gen_level(&r);
                off += 256;
            }
            if (cbpc != 0) {
                for (int k = 0; k < 16; ++k) levels[off + k] = gen_level(&r);
                off += 16;
            }
        } else {
            if (cbpc == 2) {
                for (int k = 0; k < 128; ++k) levels[off + k] = (k % 16 == 0) ? 0 : gen_level(&r);
                off += 128;
            }
            if (i16) {
                for (int k = 0; k < 16; ++k) levels[off + k] = gen_level(&r);
                off += 16;
            }
            if (cbpc != 0) {
                for (int k = 0; k < 8; ++k) levels[off + k] = gen_level(&r);
                off += 8;
            }
        }
        /* 4:4:4: the Cb and Cr planes' luma-like blocks (the same coded 8x8 blocks, their own
           levels; decode_one_component, decoder.cc:65-79); cbp_blks stays the luma plane's
           (the reference's bS reads cbp_blks[0] only, deblock.cc:135,212) */
        for (int pl = 1; f444 && pl <= 2; ++pl) {
            for (int b8 = 0; b8 < 4; ++b8) {
                if (!(cbpl & (1 << b8))) continue;
                for (int k = 0; k < 64; ++k) levels[off + k] = (i16 && (k % 16) == 0 && !t8) ? 0 : gen_level(&r);
                off += 64;
            }
            if (i16) {
                for (int k = 0; k < 16; ++k) levels[off + k] = gen_level(&r);
                off += 16;
            }
        }
        m->cbp_blks = blks;
    }
    *n_levels = off;
    return H264R_OK;
}

/* ------------------------------------------------------------ reference pictures */
static uint32_t hash3(uint64_t seed, int a, int b)
{
    rng_t r = {seed ^ ((uint64_t)(uint32_t)a << 32) ^ (uint64_t)(uint32_t)b * 0x9E3779B1ull};
    return (uint32_t)next64(&r);
}

static void texture(uint64_t seed, uint8_t* img, int w, int h, int cell)
{
    /* value noise: random lattice every `cell` pixels, bilinear (integer) + small noise */
    for (int y = 0; y < h; ++y) {
        int gy = y / cell, fy = y % cell;
        for (int x = 0; x < w; ++x) {
            int gx = x / cell, fx = x % cell;
            int v00 = hash3(seed, gx, gy) & 255, v10 = hash3(seed, gx + 1, gy) & 255;
            int v01 = hash3(seed, gx, gy + 1) & 255, v11 = hash3(seed, gx + 1, gy + 1) & 255;
            int top = v00 * (cell - fx) + v10 * fx, bot = v01 * (cell - fx) + v11 * fx;
            int v = (top * (cell - fy) + bot * fy) / (cell * cell);
            v += (int)(hash3(seed ^ 0x5bd1e995ull, x, y) % 9) - 4;
            img[y * w + x] = (uint8_t)clip3i(0, 255, v);
        }
    }
}

int h264r_synth_refpic(uint64_t seed, int slot, int width_mbs, int height_mbs, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!y || !u || !v || width_mbs <= 0 || height_mbs <= 0) return H264R_EINVAL;
    uint64_t s = seed * 31 + (uint64_t)slot * 0x2545F4914F6CDD1Dull;
    texture(s, y, width_mbs * 16, height_mbs * 16, 8);
    texture(s + 1, u, width_mbs * 8, height_mbs * 8, 4);
    texture(s + 2, v, width_mbs * 8, height_mbs * 8, 4);
    return H264R_OK;
}

int h264r_synth_refpic_fmt(uint64_t seed, int slot, int width_mbs, int height_mbs, int chroma_format, uint8_t* y,
                           uint8_t* u, uint8_t* v)
{
    const int f400 = chroma_format == H264R_SYNTH_CHROMA_400;
    if (!f400 && chroma_format != 2 && chroma_format != 3)
        return h264r_synth_refpic(seed, slot, width_mbs, height_mbs, y, u, v);
    if (!y || (!f400 && (!u || !v)) || width_mbs <= 0 || height_mbs <= 0) return H264R_EINVAL;
    uint64_t s = seed * 31 + (uint64_t)slot * 0x2545F4914F6CDD1Dull;
    if (f400) {                                            /* 4:0:0: the luma plane only */
        texture(s, y, width_mbs * 16, height_mbs * 16, 8);
        return H264R_OK;
    }
    const int cw = chroma_format == 3 ? 16 : 8;           /* 4:2:2: half width, full height */
    texture(s, y, width_mbs * 16, height_mbs * 16, 8);
    texture(s + 1, u, width_mbs * cw, height_mbs * 16, cw / 2);
    texture(s + 2, v, width_mbs * cw, height_mbs * 16, cw / 2);
    return H264R_OK;
}

int h264r_synth_algo_bytes(const h264r_mb* mbs, const int8_t* ref_idx, int W, int H, int64_t* rd, int64_t* wr)
{
    if (!mbs || !ref_idx || !rd || !wr) return H264R_EINVAL;
    int64_t R = 0, Wb = 0;
    int W4 = W * 4, plane = W4 * H * 4;
    for (int a = 0; a < W * H; ++a) {
        const h264r_mb* m = &mbs[a];
        R += 32; Wb += 384;
        if (m->mb_type == H264R_I_PCM) { R += 384; continue; }
        int cbpl = m->cbp & 15, cbpc = m->cbp >> 4;
        R += 128 * __builtin_popcount((unsigned)cbpl);
        if (m->mb_type == H264R_I_16x16) R += 32;
        if (cbpc) R += 16;
        if (cbpc == 2) R += 256;
        if (!(m->flags & H264R_MBF_INTRA)) {
            int x = a % W, y = a / W, lists = 0;
            for (int l = 0; l < 2; ++l) {
                int used = 0;
                for (int j = 0; j < 4 && !used; ++j)
                    for (int i = 0; i < 4; ++i)
                        if (ref_idx[l * plane + (y * 4 + j) * W4 + x * 4 + i] >= 0) { used = 1; break; }
                lists += used;
            }
            R += (80 + 384) * lists;
        }
    }
    *rd = R; *wr = Wb;
    return H264R_OK;
}
