// k_recon.hip -- k_inter: every MB of a batch, fully parallel, one 64-lane
// workgroup (= one wave) per MB:
//   - the per-MB deblocking record (boundary strengths + QPs, mb_deblock.h db_info_mb)
//     for EVERY MB, so the order-dependent walk of k_deblock_pic loads 48 B per MB;
//   - inter MBs and I_PCM reconstructed (mb_recon.h inter_mb / pcm_mb);
//   - intra MBs are left to k_intra_pic (they depend on their neighbours).
#include "mb_recon.h"
#include "mb_deblock.h"

using namespace h264r;

extern "C" __global__ __launch_bounds__(64) void k_inter(h264r_batch b, DbInfo* dbinfo)
{
    __shared__ ResLds R;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.y, a = blockIdx.x, lane = threadIdx.x;
    db_info_mb(b, g, pic, a, lane, dbinfo + (size_t)pic * g.nmb + a);
    inter_mb(b, g, pic, a, lane, R);
}
