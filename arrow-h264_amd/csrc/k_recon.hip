// k_recon.hip -- the fully parallel part of a batch.
//
// k_prep   one lane per 4x4 block: resolves ref_idx to the DPB slot of
//          RefPicList[l][ref_idx] (get_ref_pic dpb.cc:1046-1054 via the MB's
//          slice) and packs {mv, ref_idx | slot << 8} per list, so the per-MB
//          kernels never chase record -> slice -> slot -> plane.
// k_inter4 four MBs per wave, one lane per 4x4 block: inter MBs and I_PCM
//          reconstructed (mb_inter4.h), and the per-MB deblocking record DbInfo of
//          every MB; intra MBs are left to the intra kernels (they depend on their
//          neighbours).
#include "mb_inter4.h"

using namespace h264r;

extern "C" __global__ __launch_bounds__(256) void k_prep(h264r_batch b, uint2* __restrict__ mot, int2 rows)
{
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int idx = rows.x * 4 * g.W4 + blockIdx.x * 256 + threadIdx.x, pic = blockIdx.y;
    if (idx >= rows.y * 4 * g.W4) return;
    const int bx4 = idx % g.W4, by4 = idx / g.W4;
    const h264r_mb* mb = &b.mbs[(size_t)pic * g.nmb + (by4 >> 2) * g.wmb + (bx4 >> 2)];
    const h264r_slice* sl = &b.slices[(size_t)pic * b.slice_stride + mb->slice];
    const size_t base = (size_t)pic * 2 * g.motion_plane;
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        const int ri = b.ref_idx[base + (size_t)l * g.motion_plane + idx];
        const uint32_t mv = b.mv[base + (size_t)l * g.motion_plane + idx];
        const int slot = ri >= 0 && ri < H264R_MAX_REFS ? sl->ref_slot[l][ri] : -1;
        mot[base + (size_t)l * g.motion_plane + idx] = make_uint2(mv, (uint32_t)(uint8_t)ri | ((uint32_t)(uint8_t)slot << 8));
    }
}

// k_inter4: inter / I_PCM MBs and the deblocking record of every MB, four MBs per
// wave, one lane per 4x4 block (mb_inter4.h).  Grid (ceil(nmb / 16), pictures).
#ifndef H264R_INTER_WAVES
#define H264R_INTER_WAVES 1                 // minimum waves per SIMD asked of the register allocator
#endif
extern "C" __global__ __launch_bounds__(256, H264R_INTER_WAVES) void k_inter4(h264r_batch b, const uint2* __restrict__ mot, DbInfo* dbinfo,
                                                           int2 rows)
{
    __shared__ Inter4Lds S;
    if (threadIdx.x < 3 * H264R_MAX_SLOTS) S.planes[threadIdx.x] = b.ref_planes[threadIdx.x];
    __syncthreads();
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.y, lane = threadIdx.x & 63;
    const int a0 = rows.x * g.wmb + (blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 4;
    const int aend = rows.y * g.wmb;
    if (a0 >= aend) return;
    inter4_mbs(b, g, pic, a0, aend, lane, mot + (size_t)pic * 2 * g.motion_plane, dbinfo + (size_t)pic * g.nmb, S);
}
