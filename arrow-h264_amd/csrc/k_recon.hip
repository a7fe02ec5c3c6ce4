// k_recon.hip -- the fully parallel part of a batch.
//
// k_inter4r four MBs per wave, one lane per 4x4 block: the per-MB deblocking record DbInfo of
//           every MB (mb_inter4.h dbinfo_block), then inter MBs and I_PCM reconstructed
//           (mb_inter4.h); intra MBs are left to the intra kernels (they depend on their
//           neighbours).  Motion is read as the parser left it ({mv, ref_idx} per list) and
//           RefPicList[l][ref_idx] resolved to a DPB slot through an LDS copy of the
//           picture's slice tables.
#include "launch_cfg.h"
#include "mb_inter4.h"

using namespace h264r;

// minimum waves per SIMD asked of the register allocator: k_inter4r 4 (<= 128 VGPRs, its
// natural size with the residual loaded after the motion compensation)
#ifndef H264R_INTER_WAVES
#define H264R_INTER_WAVES 4
#endif
// The workgroup's copy of the DPB plane table and of picture `pic`'s slice ref tables, slice
// types and slice headers.  Every thread issues its loads first (clamped indices, no branch)
// and writes LDS after: three loads in flight instead of one round trip per table.
struct LdsRegs {
    const uint8_t* plane;
    uint2 refs, hdr;
};
DEV LdsRegs inter4_lds_load(const h264r_batch& b, int pic)
{
    const int t = threadIdx.x;
    const int nsl = min(b.slice_stride, INTER4_LDS_SLICES);
    const h264r_slice* sl = b.slices + (size_t)pic * b.slice_stride;
    LdsRegs r;
    // the batch's one DPB table, or picture pic's own (ref_planes_stride, include/h264r.h)
    r.plane = b.ref_planes[(size_t)pic * b.ref_planes_stride + min(t, 3 * H264R_MAX_SLOTS - 1)];
    const int ri = min(t, nsl * 4 - 1);                      // ref tables: 32 bytes per slice, 8 per thread
    r.refs = *reinterpret_cast<const uint2*>(&sl[ri >> 2].ref_slot[0][0] + 8 * (ri & 3));
    r.hdr = *reinterpret_cast<const uint2*>(&sl[min(t, nsl - 1)]);
    return r;
}
DEV void inter4_lds_store(const h264r_batch& b, const LdsRegs& r, Inter4Lds& S)
{
    const int t = threadIdx.x;
    const int nsl = min(b.slice_stride, INTER4_LDS_SLICES);
    if (t < 3 * H264R_MAX_SLOTS) S.planes[t] = r.plane;
    if (t < nsl * 4) *reinterpret_cast<uint2*>(&S.ref_slot[t >> 2][0][0] + 8 * (t & 3)) = r.refs;
    if (t < nsl) {
        S.hdr[t] = r.hdr;
        S.slice_type[t] = (uint8_t)(r.hdr.x & 255);
    }
}
DEV void inter4_lds(const h264r_batch& b, int pic, Inter4Lds& S) { inter4_lds_store(b, inter4_lds_load(b, pic), S); }

// The 16-MB groups [grp, gend) of one k_inter4r workgroup: XCD-aware (below),
// `per` (H264R_INTER_GROUPS, launch_cfg.h) consecutive groups of its
// XCD's band per workgroup, so that the workgroup's LDS tables are filled once for several
// groups.
DEV bool inter4_groups(const Geom& g, int2 rows, int per, int& grp, int& gend)
{
    const int groups = (g.wmb * (rows.y - rows.x) + 15) / 16, gb = (groups + 7) / 8;
    const int band = blockIdx.x & 7;
    grp = band * gb + (blockIdx.x >> 3) * per;
    gend = min(min(grp + per, (band + 1) * gb), groups);
    return grp < gend;
}

// k_inter4r: per 16-MB group of a workgroup, first the deblocking records DbInfo of the group's
// MBs (dbinfo_block: their neighbour records and motion are loaded with the group's own record and
// motion), then the reconstruction of its inter and I_PCM MBs (inter4_mbs); the records' registers
// are dead before the motion compensation starts (126 VGPRs, 4 waves/SIMD).  Round 6 folded the
// records' own kernel (k_dbinfo, 1.2 ms per 1024 config-3 pictures at 8 waves/SIMD) into it:
// config 3 11.96 -> 11.78 ms, config 4 4.64 -> 4.53 ms; all-intra config 2 13.87 -> 14.15 ms
// (its records now run at 4 waves/SIMD; profiles/r06_e_fused_dbinfo_ab.txt).
// It also zeroes the launch sequence's sync words and level counters (zero[0 .. nz), zero2[0 ..
// nz2)) for the kernels after it -- no memset launches per batch (the latency chain paid ~20 us
// for them, profiles/r05_ac_latency_kernels.txt).
// sp_flag: set to the launch tag when an inter MB of an SP slice was met (k_inter_sp then runs; a
// tag, not a flag, so nothing has to zero it between launch sequences -- it lies outside the
// words this kernel zeroes).
// Grid (8 * ceil(groups / (8 * per)), pictures), XCD-aware: workgroups go round-robin to the 8
// XCDs in launch order, so blockIdx.x % 8 is the XCD and it takes the 16-MB groups of band
// blockIdx.x % 8 (one eighth of the MB rows) of every picture: an XCD's motion
// compensation reads only its band of the reference pictures (+ the MV reach), which its
// 4 MB L2 holds, instead of every XCD streaming whole references through its L2.
extern "C" __global__ __launch_bounds__(256, H264R_INTER_WAVES) void k_inter4r(h264r_batch b, DbInfo* dbinfo, int2 rows,
                                                                               int* sp_flag, uint8_t* recon, int tag,
                                                                               int* zero, int nz, int* zero2, int nz2)
{
    {
        const int nt = (int)(gridDim.x * gridDim.y * blockDim.x);
        const int t = (int)((blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x);
        for (int i = t; i < nz; i += nt) zero[i] = 0;
        for (int i = t; i < nz2; i += nt) zero2[i] = 0;
    }
    __shared__ Inter4Lds S;
    __shared__ DbTables T;
    const int pic = blockIdx.y;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    int grp, gend;
    if (!inter4_groups(g, rows, H264R_INTER_GROUPS, grp, gend)) return;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int aend = rows.y * g.wmb;
    const h264r_slice* slices = b.slices + (size_t)pic * b.slice_stride;
    int a0 = rows.x * g.wmb + (grp * 4 + wave) * 4;
    const uint2 tv = db_tables_load(threadIdx.x);
    Inter4Pre pre = inter4_pre(b, g, pic, a0, aend, lane);
    DbNb nb = dbinfo_pre(b, g, pic, a0, aend, lane);
    const LdsRegs lr = inter4_lds_load(b, pic);
    db_tables_store(T, threadIdx.x, tv);
    inter4_lds_store(b, lr, S);
    __syncthreads();
    for (;;) {
        if (a0 >= aend) return;
        {
            const int a = a0 + (lane >> 4);
            const bool valid = a < aend;
            const int aa = valid ? a : aend - 1;
            const uint2 m0 = motion_word(pre.mv[0], pre.ri[0], slices, S, pre.q.slice, 0);
            const uint2 m1 = motion_word(pre.mv[1], pre.ri[1], slices, S, pre.q.slice, 1);
            if (!(H264R_INTER_DIAG & 32))
                dbinfo_block(b, g, pic, aa, valid, lane & 15, S, T, pre.q, m0, m1, slice_hdr(slices, S, pre.q.slice), nb,
                             dbinfo + (size_t)pic * g.nmb);
        }
        int ln = lane;
        asm volatile("" : "+v"(ln));
        inter4_mbs<false>(b, g, pic, a0, aend, ln, S, sp_flag, pre, recon, tag);
        if (++grp >= gend) return;
        a0 = rows.x * g.wmb + (grp * 4 + wave) * 4;
        int ln2 = lane;
        asm volatile("" : "+v"(ln2));
        pre = inter4_pre(b, g, pic, a0, aend, ln2);
        nb = dbinfo_pre(b, g, pic, a0, aend, ln2);
    }
}


// k_inter_sp: the inter MBs of SP slices (inverse_transform_sp), after k_inter4.  A
// persistent grid that leaves at once unless k_inter4 set sp_flag (so a batch without SP
// slices pays one short launch), then strides over (16-MB group, picture).
extern "C" __global__ __launch_bounds__(256) void k_inter_sp(h264r_batch b, int2 rows, const int* sp_flag, uint8_t* recon,
                                                             int tag)
{
    if (__hip_atomic_load(sp_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag) return;
    __shared__ Inter4Lds S;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int groups = (g.wmb * (rows.y - rows.x) + 15) / 16;
    const int aend = rows.y * g.wmb;
    for (int w = blockIdx.x; w < groups * b.num_pics; w += gridDim.x) {
        const int pic = w / groups, grp = w % groups;
        __syncthreads();                              // the previous item's readers are done with S
        inter4_lds(b, pic, S);
        __syncthreads();
        const int a0 = rows.x * g.wmb + (grp * 4 + wave) * 4;
        if (a0 < aend) inter4_mbs<true>(b, g, pic, a0, aend, lane, S, nullptr, inter4_pre(b, g, pic, a0, aend, lane), recon, 0);
    }
}

// k_untile: the MB-tiled reconstruction copied into the output planes as it stands (the
// launch sequence without deblocking, H264R_DBG_NO_DEBLOCK).  One thread per luma row
// (16 B) or chroma row (8 B) of an MB: 32 per MB.  Grid (ceil(32 * MBs / 256), pictures).
extern "C" __global__ __launch_bounds__(256) void k_untile(h264r_batch b, int2 rows, const uint8_t* __restrict__ recon)
{
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.y;
    const int t = blockIdx.x * 256 + threadIdx.x, a = rows.x * g.wmb + (t >> 5), k = t & 31;
    if (a >= rows.y * g.wmb) return;
    const int mbx = a % g.wmb, mby = a / g.wmb;
    const uint8_t* mb = recon + ((size_t)pic * g.nmb + a) * RECON_MB;
    if (k < 16) {
        *reinterpret_cast<uint4*>(b.out_y + (size_t)pic * g.ysz + (size_t)(mby * 16 + k) * g.W + mbx * 16) =
            *reinterpret_cast<const uint4*>(mb + k * 16);
    } else {
        const int pl = (k - 16) >> 3, r = k & 7;
        uint8_t* dst = (pl ? b.out_v : b.out_u) + (size_t)pic * g.csz + (size_t)(mby * 8 + r) * g.Wc + mbx * 8;
        *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(mb + RECON_CB + pl * 64 + r * 8);
    }
}

// k_derive444: one colour plane `pl` of a 4:4:4 batch as a 4:2:0-shaped batch whose luma is that
// plane (h264r_host.hip run_444; decode_one_component decoder.cc:65-79 runs the luma path on each
// plane of a ChromaArrayType 3 MB):
//   records: qp_y := QpC[pl - 1] (deblocking, deblock.cc:469-470), qp_scaled[0] := qp_scaled[pl]
//            (dequantisation, transform.cc:400-401), coef_off := the plane's luma-like level block
//            (include/h264r.h, 4:4:4), CodedBlockPatternChroma 0, chroma mode DC; cbp_blks stays
//            the luma plane's (the bS reads cbp_blks[0] only, deblock.cc:135,212);
//   slices:  the plane's weights and offsets in the luma slots, the chroma denominator
//            (mc_prediction inter_prediction.cc:68-74);
//   quant:   the plane's 4x4 and 8x8 lists in the luma slots (set_quant transform.cc:259-301);
//   DPB tables: every plane entry of a slot -> the slot's plane pl (the luma MC reads it; the
//            derived chroma reads stay inside it).
// Field pictures and SP slices are not on the 4:4:4 / 4:2:2 / 4:0:0 paths: such a batch flags the
// device error word.  qpl: the plane whose lists and DPB planes the pass takes -- pl, except for a
// separate-colour-plane (JV) batch: its monochrome records are taken as they are (pl 0) and its
// lists and references are those of colour plane qpl (transform.cc:402, inter_prediction.cc:175-177).
extern "C" __global__ __launch_bounds__(256) void k_derive444(h264r_batch b, int pl, int qpl, h264r_mb* __restrict__ mbs,
                                                              h264r_slice* __restrict__ slices, h264r_quant* __restrict__ quant,
                                                              const uint8_t** __restrict__ refs, int ntab, int* err)
{
    const int64_t nt = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nmb = (int64_t)b.width_mbs * b.height_mbs, P = b.num_pics;
    for (int64_t i = t0; i < P * nmb; i += nt) {
        h264r_mb m = b.mbs[i];
        const int cbpl = m.cbp & 15;
        if (m.mb_type == H264R_I_PCM) m.coef_off += 128u * (uint32_t)pl;
        else m.coef_off += (uint32_t)(pl * (64 * __builtin_popcount(cbpl) + (m.mb_type == H264R_I_16x16 ? 16 : 0)));
        if (pl) { m.qp_y = m.qp_c[pl - 1]; m.qp_scaled[0] = m.qp_scaled[pl]; }
        m.cbp = (uint8_t)cbpl;
        m.chroma_mode = 0;
        mbs[i] = m;
    }
    for (int64_t i = t0; i < P * b.slice_stride; i += nt) {
        h264r_slice x = b.slices[i];
        if (x.slice_type == H264R_SLICE_SP) atomicOr(err, 4);     // SP slices: 4:2:0 only (Extended profile)
        if (pl) {
            for (int l = 0; l < 2; ++l)
                for (int r = 0; r < H264R_MAX_REFS; ++r) {
                    x.wp_weight[l][r][0] = x.wp_weight[l][r][pl];
                    x.wp_offset[l][r][0] = x.wp_offset[l][r][pl];
                }
            x.luma_log2_wd = x.chroma_log2_wd;
        }
        slices[i] = x;
    }
    constexpr int QW = (int)(sizeof(h264r_quant) / 2);          // int16 entries of a table
    constexpr int S4 = 3 * 6 * 16, S8 = 3 * 6 * 64;              // one intra/inter half of each array
    for (int64_t i = t0; i < P * QW; i += nt) {
        const int64_t q = i / QW;
        int k = (int)(i % QW);
        const int16_t* src = reinterpret_cast<const int16_t*>(b.quant + q);
        // the luma slot [intra/inter][0] takes plane pl's entry; everything else is copied
        int from = k;
        if (k < 2 * S4) {
            const int half = k / S4, r = k % S4;
            if (r < 6 * 16) from = half * S4 + qpl * 6 * 16 + r;
        } else {
            const int k8 = k - 2 * S4, half = k8 / S8, r = k8 % S8;
            if (r < 6 * 64) from = 2 * S4 + half * S8 + qpl * 6 * 64 + r;
        }
        reinterpret_cast<int16_t*>(quant + q)[k] = src[from];
    }
    for (int64_t i = t0; i < (int64_t)ntab * 3 * H264R_MAX_SLOTS; i += nt) {
        const int64_t tab = i / (3 * H264R_MAX_SLOTS), e = i % (3 * H264R_MAX_SLOTS), slot = e / 3;
        refs[i] = b.ref_planes[tab * b.ref_planes_stride + 3 * slot + qpl];
    }
    for (int64_t i = t0; i < P; i += nt)
        if (b.pics[i].structure != H264R_FRAME) atomicOr(err, 1);
}
