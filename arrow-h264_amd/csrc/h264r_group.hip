// h264r_group.hip -- include/h264r_group.h: the exchange of slice bands between the ranks of a
// multi-GPU job.
//
// One exchange = pack (k_band_copy: the rows every peer needs, of every picture, into one
// contiguous segment per peer) -> transfers (RCCL ncclSend / ncclRecv in one group, or the
// caller's transport) -> unpack (k_band_copy back into the planes).  With RCCL all three are
// enqueued on the caller's stream: no host synchronisation, the next decode on that stream reads
// the received rows.  RCCL is loaded with dlopen when the first group is made.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "h264r.h"
#include "h264r_group.h"

namespace {

// One segment of a staging buffer: rows [r0, r1) of every picture for one peer; `pre` = the rows
// of the segments before it, so that its offset is pre * num_pics * (bytes of one MB row).
struct SegDev { int32_t r0, r1, pre, peer; };

// One thread moves 8 bytes (MB rows are 256 W / 64 W bytes: multiples of 8).  Grid: x = chunks of
// one picture's part of a segment, y = picture, z = segment.
__global__ void __launch_bounds__(256) k_band_copy(const SegDev* __restrict__ segs, int nk, uint8_t* __restrict__ buf,
                                                   uint8_t* y, uint8_t* u, uint8_t* v, int64_t sy, int64_t sc,
                                                   int64_t rby, int64_t rbc, int unpack)
{
    const SegDev s = segs[blockIdx.z];
    const int64_t rows = s.r1 - s.r0;
    const int64_t ny = rows * rby, nc = rows * rbc, per = ny + 2 * nc;
    const int64_t pic = blockIdx.y;
    uint8_t* seg = buf + (int64_t)s.pre * nk * (rby + 2 * rbc) + pic * per;
    for (int64_t o = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; o < per;
         o += (int64_t)gridDim.x * blockDim.x * 8) {
        uint8_t* pl;
        if (o < ny) pl = y + pic * sy + s.r0 * rby + o;
        else if (o < ny + nc) pl = u + pic * sc + s.r0 * rbc + (o - ny);
        else pl = v + pic * sc + s.r0 * rbc + (o - ny - nc);
        uint64_t* a = reinterpret_cast<uint64_t*>(pl);
        uint64_t* b = reinterpret_cast<uint64_t*>(seg + o);
        if (unpack) *a = *b;
        else *b = *a;
    }
}

struct Rccl {
    bool ok = false;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) gstart = nullptr;
    decltype(&ncclGroupEnd) gend = nullptr;
};

// The RCCL a process already holds (torch's, when torch is loaded) is found by its SONAME first.
const Rccl& rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* env = getenv("H264R_RCCL");
        const char* names[] = {env, "librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        void* h = nullptr;
        for (const char* n : names)
            if (n && *n && (h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
        if (!h) return;
        r.get_id = reinterpret_cast<decltype(r.get_id)>(dlsym(h, "ncclGetUniqueId"));
        r.init = reinterpret_cast<decltype(r.init)>(dlsym(h, "ncclCommInitRank"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
        r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
        r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
        r.gstart = reinterpret_cast<decltype(r.gstart)>(dlsym(h, "ncclGroupStart"));
        r.gend = reinterpret_cast<decltype(r.gend)>(dlsym(h, "ncclGroupEnd"));
        r.ok = r.get_id && r.init && r.destroy && r.send && r.recv && r.gstart && r.gend;
    });
    return r;
}

bool valid_bands(int nranks, const int32_t* bands)
{
    if (nranks < 1 || nranks > H264R_GROUP_MAX_RANKS || !bands) return false;
    for (int r = 0; r < nranks; ++r)
        if (bands[2 * r] < 0 || bands[2 * r + 1] < 0) return false;
    return true;
}

}  // namespace

struct h264r_group {
    int device = -1, nranks = 1, rank = 0;
    bool use_rccl = false;
    ncclComm_t comm = nullptr;
    h264r_transport t{};
    // plan
    int W = 0, H = 0, max_pics = 0;
    std::vector<SegDev> give, need;      // peers with rows, increasing rank order
    int give_rows = 0, need_rows = 0;
    SegDev* d_segs = nullptr;            // give then need
    uint8_t *d_send = nullptr, *d_recv = nullptr, *h_send = nullptr, *h_recv = nullptr;
    bool host_pinned = false;
    int64_t sent = 0, received = 0, transfers = 0;

    int64_t mbrow() const { return 384LL * W; }
    void free_buffers()
    {
        if (device >= 0) {
            (void)hipSetDevice(device);
            if (d_segs) (void)hipFree(d_segs);
            if (d_send) (void)hipFree(d_send);
            if (d_recv) (void)hipFree(d_recv);
        }
        if (host_pinned) {
            if (h_send) (void)hipHostFree(h_send);
            if (h_recv) (void)hipHostFree(h_recv);
        } else {
            free(h_send);
            free(h_recv);
        }
        d_segs = nullptr; d_send = d_recv = h_send = h_recv = nullptr;
    }
};

extern "C" {

int h264r_group_plan(int nranks, int rank, const int32_t* bands, int mode, int halo_mb_rows, int32_t* need,
                     int32_t* give)
{
    if (!valid_bands(nranks, bands) || rank < 0 || rank >= nranks || !need || !give || halo_mb_rows < 0 ||
        (mode != H264R_XCHG_HALO && mode != H264R_XCHG_ALLGATHER))
        return H264R_EINVAL;
    const int b0 = bands[2 * rank], b1 = bands[2 * rank + 1];
    for (int r = 0; r < nranks; ++r) {
        need[2 * r] = need[2 * r + 1] = give[2 * r] = give[2 * r + 1] = 0;
        const int r0 = bands[2 * r], r1 = bands[2 * r + 1];
        if (r == rank) continue;
        if (mode == H264R_XCHG_ALLGATHER) {
            if (r1 > r0) { need[2 * r] = r0; need[2 * r + 1] = r1; }
            if (b1 > b0) { give[2 * r] = b0; give[2 * r + 1] = b1; }
            continue;
        }
        if (b1 <= b0 || r1 <= r0) continue;
        const int n0 = std::max(b0 - halo_mb_rows, r0), n1 = std::min(b1 + halo_mb_rows, r1);
        if (n1 > n0) { need[2 * r] = n0; need[2 * r + 1] = n1; }
        const int g0 = std::max(r0 - halo_mb_rows, b0), g1 = std::min(r1 + halo_mb_rows, b1);
        if (g1 > g0) { give[2 * r] = g0; give[2 * r + 1] = g1; }
    }
    return H264R_OK;
}

int h264r_group_unique_id(uint8_t id[H264R_GROUP_ID_BYTES])
{
    if (!id) return H264R_EINVAL;
    const Rccl& R = rccl();
    if (!R.ok) return H264R_ENODEVICE;
    ncclUniqueId u;
    if (R.get_id(&u) != ncclSuccess) return H264R_EDEVICE;
    static_assert(sizeof(u) == H264R_GROUP_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof u);
    return H264R_OK;
}

static int make_group(h264r_group** out, int device, int nranks, int rank)
{
    if (!out || nranks < 1 || nranks > H264R_GROUP_MAX_RANKS || rank < 0 || rank >= nranks) return H264R_EINVAL;
    *out = nullptr;
    if (device >= 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || device >= n) return H264R_ENODEVICE;
        if (hipSetDevice(device) != hipSuccess) return H264R_EDEVICE;
    }
    h264r_group* g = new (std::nothrow) h264r_group;
    if (!g) return H264R_ENOMEM;
    g->device = device;
    g->nranks = nranks;
    g->rank = rank;
    *out = g;
    return H264R_OK;
}

int h264r_group_create(h264r_group** out, int device, int nranks, int rank, const uint8_t id[H264R_GROUP_ID_BYTES])
{
    if (!id || device < 0) return H264R_EINVAL;
    const Rccl& R = rccl();
    if (!R.ok) return H264R_ENODEVICE;
    int st = make_group(out, device, nranks, rank);
    if (st != H264R_OK) return st;
    h264r_group* g = *out;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    if (R.init(&g->comm, nranks, u, rank) != ncclSuccess) {
        delete g;
        *out = nullptr;
        return H264R_EDEVICE;
    }
    g->use_rccl = true;
    return H264R_OK;
}

int h264r_group_create_transport(h264r_group** out, int device, int nranks, int rank, const h264r_transport* t)
{
    if (!t || !t->start || !t->send || !t->recv || !t->finish) return H264R_EINVAL;
    int st = make_group(out, device, nranks, rank);
    if (st == H264R_OK) (*out)->t = *t;
    return st;
}

int h264r_group_destroy(h264r_group* g)
{
    if (!g) return H264R_EINVAL;
    g->free_buffers();
    if (g->comm) rccl().destroy(g->comm);
    delete g;
    return H264R_OK;
}

int h264r_group_set_bands(h264r_group* g, int width_mbs, int height_mbs, const int32_t* bands, int mode,
                          int halo_mb_rows, int max_pics)
{
    if (!g || width_mbs < 1 || height_mbs < 1 || max_pics < 1 || max_pics > 65535 || !valid_bands(g->nranks, bands))
        return H264R_EINVAL;
    for (int r = 0; r < g->nranks; ++r)
        if (bands[2 * r + 1] > height_mbs) return H264R_EINVAL;
    std::vector<int32_t> need(2 * g->nranks), give(2 * g->nranks);
    int st = h264r_group_plan(g->nranks, g->rank, bands, mode, halo_mb_rows, need.data(), give.data());
    if (st != H264R_OK) return st;
    g->free_buffers();
    g->W = width_mbs;
    g->H = height_mbs;
    g->max_pics = max_pics;
    g->give.clear();
    g->need.clear();
    g->give_rows = g->need_rows = 0;
    for (int r = 0; r < g->nranks; ++r) {
        if (give[2 * r + 1] > give[2 * r]) {
            g->give.push_back({give[2 * r], give[2 * r + 1], g->give_rows, r});
            g->give_rows += give[2 * r + 1] - give[2 * r];
        }
        if (need[2 * r + 1] > need[2 * r]) {
            g->need.push_back({need[2 * r], need[2 * r + 1], g->need_rows, r});
            g->need_rows += need[2 * r + 1] - need[2 * r];
        }
    }
    const size_t sbytes = (size_t)max_pics * g->give_rows * g->mbrow(), rbytes = (size_t)max_pics * g->need_rows * g->mbrow();
    const size_t nseg = g->give.size() + g->need.size();
    if (g->device >= 0) {
        (void)hipSetDevice(g->device);
        if ((nseg && hipMalloc(reinterpret_cast<void**>(&g->d_segs), nseg * sizeof(SegDev)) != hipSuccess) ||
            (sbytes && hipMalloc(reinterpret_cast<void**>(&g->d_send), sbytes) != hipSuccess) ||
            (rbytes && hipMalloc(reinterpret_cast<void**>(&g->d_recv), rbytes) != hipSuccess)) {
            g->free_buffers();
            return H264R_ENOMEM;
        }
        std::vector<SegDev> all(g->give);
        all.insert(all.end(), g->need.begin(), g->need.end());
        if (nseg && hipMemcpy(g->d_segs, all.data(), nseg * sizeof(SegDev), hipMemcpyHostToDevice) != hipSuccess) {
            g->free_buffers();
            return H264R_EDEVICE;
        }
    }
    if (!g->use_rccl) {     // the callback transport sends host buffers
        g->host_pinned = g->device >= 0;
        if (g->host_pinned) {
            if ((sbytes && hipHostMalloc(reinterpret_cast<void**>(&g->h_send), sbytes, hipHostMallocDefault) != hipSuccess) ||
                (rbytes && hipHostMalloc(reinterpret_cast<void**>(&g->h_recv), rbytes, hipHostMallocDefault) != hipSuccess)) {
                g->free_buffers();
                return H264R_ENOMEM;
            }
        } else if ((sbytes && !(g->h_send = static_cast<uint8_t*>(malloc(sbytes)))) ||
                   (rbytes && !(g->h_recv = static_cast<uint8_t*>(malloc(rbytes))))) {
            g->free_buffers();
            return H264R_ENOMEM;
        }
    }
    return H264R_OK;
}

// Host form of k_band_copy (planes in host memory, callback transport).
static void host_copy(const h264r_group* g, const std::vector<SegDev>& segs, int nk, uint8_t* buf, uint8_t* const pl[3],
                      const int64_t stride[3], bool unpack)
{
    const int64_t rb[3] = {256LL * g->W, 64LL * g->W, 64LL * g->W};
    for (const SegDev& s : segs) {
        const int64_t rows = s.r1 - s.r0;
        uint8_t* seg = buf + (int64_t)s.pre * nk * g->mbrow();
        for (int i = 0; i < nk; ++i)
            for (int k = 0; k < 3; ++k) {
                uint8_t* p = pl[k] + i * stride[k] + s.r0 * rb[k];
                const int64_t n = rows * rb[k];
                if (unpack) memcpy(p, seg, n);
                else memcpy(seg, p, n);
                seg += n;
            }
    }
}

int h264r_group_exchange(h264r_group* g, int num_pics, uint8_t* y, uint8_t* u, uint8_t* v, int64_t stride_y,
                         int64_t stride_c, void* stream)
{
    if (!g || !g->max_pics) return g ? H264R_ESTATE : H264R_EINVAL;
    const int64_t W = g->W, H = g->H;
    if (num_pics < 1 || num_pics > g->max_pics || !y || !u || !v || stride_y < 256 * W * H || stride_c < 64 * W * H)
        return H264R_EINVAL;
    // k_band_copy moves 8-byte words
    if (g->device >= 0 && (((uintptr_t)y | (uintptr_t)u | (uintptr_t)v | (uint64_t)stride_y | (uint64_t)stride_c) & 7))
        return H264R_EINVAL;
    if (g->nranks == 1 || (g->give.empty() && g->need.empty())) return H264R_OK;
    const int nk = num_pics;
    const int64_t mbrow = g->mbrow();
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t sbytes = (size_t)nk * g->give_rows * mbrow, rbytes = (size_t)nk * g->need_rows * mbrow;
    uint8_t* const pl[3] = {y, u, v};
    const int64_t stride[3] = {stride_y, stride_c, stride_c};

    auto launch = [&](const SegDev* segs, size_t nseg, uint8_t* buf, int rows, int unpack) {
        if (!nseg) return hipSuccess;
        const int64_t per8 = (int64_t)rows * mbrow / 8 / (int64_t)nseg + 1;      // average 8-byte units per picture segment
        const int gx = (int)std::min<int64_t>(64, (per8 + 255) / 256);
        hipLaunchKernelGGL(k_band_copy, dim3(gx, nk, (unsigned)nseg), dim3(256), 0, s, segs, nk, buf, y, u, v, stride_y,
                           stride_c, 256 * W, 64 * W, unpack);
        return hipGetLastError();
    };

    if (g->device >= 0) {
        (void)hipSetDevice(g->device);
        if (launch(g->d_segs, g->give.size(), g->d_send, g->give_rows, 0) != hipSuccess) return H264R_EDEVICE;
    } else {
        host_copy(g, g->give, nk, g->h_send, pl, stride, false);
    }

    if (g->use_rccl) {
        const Rccl& R = rccl();
        bool ok = R.gstart() == ncclSuccess;
        for (const SegDev& sg : g->give)
            ok = ok && R.send(g->d_send + (size_t)sg.pre * nk * mbrow, (size_t)(sg.r1 - sg.r0) * nk * mbrow, ncclUint8,
                              sg.peer, g->comm, s) == ncclSuccess;
        for (const SegDev& sg : g->need)
            ok = ok && R.recv(g->d_recv + (size_t)sg.pre * nk * mbrow, (size_t)(sg.r1 - sg.r0) * nk * mbrow, ncclUint8,
                              sg.peer, g->comm, s) == ncclSuccess;
        ok = (R.gend() == ncclSuccess) && ok;
        if (!ok) return H264R_EDEVICE;
    } else {
        if (g->device >= 0) {
            if ((sbytes && hipMemcpyAsync(g->h_send, g->d_send, sbytes, hipMemcpyDeviceToHost, s) != hipSuccess) ||
                hipStreamSynchronize(s) != hipSuccess)
                return H264R_EDEVICE;
        }
        const h264r_transport& t = g->t;
        bool ok = t.start(t.user) == 0;
        for (const SegDev& sg : g->give)
            ok = ok && t.send(t.user, sg.peer, g->h_send + (size_t)sg.pre * nk * mbrow, (size_t)(sg.r1 - sg.r0) * nk * mbrow) == 0;
        for (const SegDev& sg : g->need)
            ok = ok && t.recv(t.user, sg.peer, g->h_recv + (size_t)sg.pre * nk * mbrow, (size_t)(sg.r1 - sg.r0) * nk * mbrow) == 0;
        ok = (t.finish(t.user) == 0) && ok;
        if (!ok) return H264R_EDEVICE;
        if (g->device >= 0 && rbytes &&
            hipMemcpyAsync(g->d_recv, g->h_recv, rbytes, hipMemcpyHostToDevice, s) != hipSuccess)
            return H264R_EDEVICE;
    }

    if (g->device >= 0) {
        if (launch(g->d_segs + g->give.size(), g->need.size(), g->d_recv, g->need_rows, 1) != hipSuccess)
            return H264R_EDEVICE;
        if (!g->use_rccl && hipStreamSynchronize(s) != hipSuccess) return H264R_EDEVICE;   // h_recv reused next time
    } else {
        host_copy(g, g->need, nk, g->h_recv, pl, stride, true);
    }
    g->sent += sbytes;
    g->received += rbytes;
    g->transfers += g->give.size() + g->need.size();
    return H264R_OK;
}

int h264r_group_stats(h264r_group* g, int64_t* sent, int64_t* received, int64_t* transfers)
{
    if (!g) return H264R_EINVAL;
    if (sent) *sent = g->sent;
    if (received) *received = g->received;
    if (transfers) *transfers = g->transfers;
    return H264R_OK;
}

}  // extern "C"
