// k_recon.hip -- the fully parallel part of a batch.
//
// k_inter4 four MBs per wave, one lane per 4x4 block: inter MBs and I_PCM
//          reconstructed (mb_inter4.h), and the per-MB deblocking record DbInfo of
//          every MB; intra MBs are left to the intra kernels (they depend on their
//          neighbours).  Motion is read as the parser left it ({mv, ref_idx} per list)
//          and RefPicList[l][ref_idx] resolved to a DPB slot through an LDS copy of the
//          picture's slice tables.
#include "mb_inter4.h"

using namespace h264r;

// Grid (ceil(nmb / 16), pictures).
#ifndef H264R_INTER_WAVES
#define H264R_INTER_WAVES 3                 // minimum waves per SIMD asked of the register allocator (<= 168 VGPRs)
#endif
extern "C" __global__ __launch_bounds__(256, H264R_INTER_WAVES) void k_inter4(h264r_batch b, DbInfo* dbinfo, int2 rows)
{
    __shared__ Inter4Lds S;
    const int pic = blockIdx.y;
    if (threadIdx.x < 3 * H264R_MAX_SLOTS) S.planes[threadIdx.x] = b.ref_planes[threadIdx.x];
    {
        // the picture's ref tables: 32 bytes per slice, 8 per thread
        const int nsl = min(b.slice_stride, INTER4_LDS_SLICES);
        const h264r_slice* sl = b.slices + (size_t)pic * b.slice_stride;
        for (int i = threadIdx.x; i < nsl * 4; i += blockDim.x)
            *reinterpret_cast<uint2*>(&S.ref_slot[i >> 2][0][0] + 8 * (i & 3)) =
                *reinterpret_cast<const uint2*>(&sl[i >> 2].ref_slot[0][0] + 8 * (i & 3));
    }
    __syncthreads();
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int lane = threadIdx.x & 63;
    const int a0 = rows.x * g.wmb + (blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 4;
    const int aend = rows.y * g.wmb;
    if (a0 >= aend) return;
    inter4_mbs(b, g, pic, a0, aend, lane, dbinfo + (size_t)pic * g.nmb, S);
}
