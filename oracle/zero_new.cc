/*
 * zero_new.cc -- TEST INFRASTRUCTURE ONLY: zero-filled operator new for the shim builds.
 *
 * The reference's Annex-B reader never initialises annex_b_t::nextstartcodebytes
 * (parser/bitstream.cc:150-156; get_nalu reads it first, :207).  In a fresh process the
 * heap block comes back zeroed and the decoder works; once the HIP runtime has been
 * loaded (libh264r.so) the block is recycled memory and the reader writes a garbage
 * number of zero bytes -- no frame is found and the process faults.  The shim binaries
 * (oracle/_ref/ldecod_shim, ldecod_h264r) link this file so that every `new` returns
 * zeroed memory: the behaviour of the reference in a fresh process, without editing
 * the reference's sources.  A maintainer shipping the shim would fix the member's
 * initialisation in bitstream.cc instead.
 */
#include <cstdlib>
#include <new>

void* operator new(std::size_t n)
{
    void* p = std::calloc(1, n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void* operator new[](std::size_t n) { return operator new(n); }
void* operator new(std::size_t n, const std::nothrow_t&) noexcept { return std::calloc(1, n ? n : 1); }
void* operator new[](std::size_t n, const std::nothrow_t&) noexcept { return std::calloc(1, n ? n : 1); }
void operator delete(void* p) noexcept { std::free(p); }
void operator delete[](void* p) noexcept { std::free(p); }
void operator delete(void* p, std::size_t) noexcept { std::free(p); }
void operator delete[](void* p, std::size_t) noexcept { std::free(p); }
