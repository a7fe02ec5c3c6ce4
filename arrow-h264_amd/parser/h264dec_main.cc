// h264dec_main.cc -- command-line decoder over the repo's own parser (h264p) and the h264r
// reconstruction ABI: `h264dec -i stream.264 -o out.yuv [-d device]`, the reference's
// `ldecod -i -o` (core/main.cc) for the path this repo covers.  Frames are written in output
// order, cropped to the SPS window, 8-bit planar 4:2:0, 4:2:2 or 4:4:4, or 4:0:0 with 128-valued 4:2:0 chroma (write_out_picture, output.cc:109-227).
// Linked against libh264r.so it decodes on MI355X; the test build links the CPU
// implementation of the same ABI instead (oracle/Makefile h264dec_cpu).
// `-r N`: decode the stream N more times after the written pass and print the wall time per
// frame of those passes (parse + reconstruction + readback, no file output) to stderr.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "h264p.h"
#include "h264r.h"

static int write_frame(void* user, const h264p_frame* f)
{
    FILE* out = static_cast<FILE*>(user);
    const int x0 = f->crop_left, x1 = f->width - f->crop_right;
    const int y0 = f->crop_top, y1 = f->height - f->crop_bottom;
    for (int y = y0; y < y1; ++y)
        if (fwrite(f->y + (size_t)y * f->width + x0, 1, x1 - x0, out) != (size_t)(x1 - x0)) return 1;
    if (f->chroma_format == 0) {
        // 4:0:0: two planes of 128 a quarter of the cropped luma each, as the reference's WriteUV
        // default fakes a 4:2:0 file (output.cc:205-224)
        const std::vector<uint8_t> fake((size_t)(x1 - x0) * (y1 - y0) / 4, 128);
        for (int k = 0; k < 2; ++k)
            if (fwrite(fake.data(), 1, fake.size(), out) != fake.size()) return 1;
        return 0;
    }
    // log2 SubWidthC / SubHeightC: 4:2:2 keeps every row, 4:4:4 every row and column
    const int sh = f->chroma_format == 1 ? 1 : 0, sw = f->chroma_format == 3 ? 0 : 1;
    const int cw = f->width >> sw, n = (x1 - x0) >> sw;
    for (const uint8_t* c : {f->u, f->v})
        for (int y = y0 >> sh; y < y1 >> sh; ++y)
            if (fwrite(c + (size_t)y * cw + (x0 >> sw), 1, n, out) != (size_t)n) return 1;
    return 0;
}

int main(int argc, char** argv)
{
    const char *in = nullptr, *outp = nullptr;
    int device = 0, repeat = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "-i")) in = argv[i + 1];
        else if (!strcmp(argv[i], "-o")) outp = argv[i + 1];
        else if (!strcmp(argv[i], "-d")) device = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-r")) repeat = atoi(argv[i + 1]);
    }
    if (!in || !outp) {
        fprintf(stderr, "usage: %s -i stream.264 -o out.yuv [-d device] [-r repeats]\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(in, "rb");
    if (!f) { perror(in); return 1; }
    std::vector<uint8_t> data;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + n);
    fclose(f);
    FILE* out = fopen(outp, "wb");
    if (!out) { perror(outp); return 1; }
    h264p_dec* dec = nullptr;
    int st = h264p_create(&dec, device);
    if (st == H264R_OK) st = h264p_decode(dec, data.data(), data.size(), write_frame, out);
    if (st == H264R_OK && repeat > 0) {
        long frames = 0;
        auto count = [](void* u, const h264p_frame*) { ++*static_cast<long*>(u); return 0; };
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < repeat && st == H264R_OK; ++r) st = h264p_decode(dec, data.data(), data.size(), count, &frames);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (st == H264R_OK) fprintf(stderr, "h264dec: %ld frames, %.3f ms per frame\n", frames, ms / frames);
    }
    if (st != H264R_OK)
        fprintf(stderr, "h264dec: %s (%s)\n", h264r_strerror(st), dec ? h264p_last_error(dec) : "");
    h264p_destroy(dec);
    if (fclose(out) != 0 && st == H264R_OK) st = H264R_EINVAL;
    return st == H264R_OK ? 0 : 1;
}
