// Host-side AddressSanitizer check of libisg's C-ABI (SURVEY.md §5 "sanitizers": GPU ASan
// is not available on this pool, so the host half runs instrumented on the CPU).
//
// Built by tools/asan/build.sh from every libisg source compiled host-only
// (-Xarch_host -fsanitize=address, host half only): no device code, no GPU needed. It drives the
// paths whose memory handling is host code — argument validation, the error plumbing,
// the executor's record parsing and pointer fix-ups, the chunking of host item arrays —
// with valid and malformed inputs; kernel launches fail cleanly without a device.
// Exit 0 and no ASan report = pass.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/isg.h"

static int failures = 0;
#define EXPECT(c)                                                        \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                  \
        }                                                                \
    } while (0)

// executor blob: header {kind, desc_bytes, nfix, flags}, desc (8-aligned), fixes
static void put_op(std::vector<char>& b, int kind, const void* desc, int bytes,
                   const std::vector<isg_ref>& fix, const std::vector<int>& locs, int flags = 0) {
    int32_t h[4] = {kind, bytes, (int32_t)fix.size(), flags};
    b.insert(b.end(), (char*)h, (char*)h + sizeof(h));
    b.insert(b.end(), (const char*)desc, (const char*)desc + bytes);
    b.resize(b.size() + ((8 - bytes % 8) % 8), 0);
    for (size_t i = 0; i < fix.size(); ++i) {
        int32_t lf[2] = {locs[i], fix[i].slot};
        b.insert(b.end(), (char*)lf, (char*)lf + sizeof(lf));
        b.insert(b.end(), (const char*)&fix[i].offset, (const char*)&fix[i].offset + 8);
    }
}

int main() {
    EXPECT(isg_abi_version() > 0);
    EXPECT(isg_stat_replicas() == ISG_STAT_REP);
    for (int i = 0; i <= 16; ++i) EXPECT(isg_record_size(i) > 0);
    EXPECT(isg_record_size(-1) == -1 && isg_record_size(99) == -1);

    // argument validation and the thread-local message
    isg_conv_geom g{};
    EXPECT(isg_conv_fwd(nullptr, nullptr, nullptr, nullptr, nullptr) == ISG_ERR_INVALID);
    EXPECT(std::strlen(isg_last_error()) > 0);
    g.N = 1; g.Ci = 4; g.H = 8; g.W = 8; g.Co = 4; g.OH = 9; g.OW = 8;
    g.KH = g.KW = 3; g.SH = g.SW = 1; g.PH = g.PW = 1; g.DH = g.DW = 1; g.groups = 1;
    EXPECT(isg_conv_fwd(&g, nullptr, nullptr, nullptr, nullptr) == ISG_ERR_INVALID);  // OH
    g.OH = 8;
    g.groups = 2;
    EXPECT(isg_conv_dgrad(&g, nullptr, nullptr, nullptr, nullptr) == ISG_ERR_UNSUPPORTED);
    g.groups = 1;
    EXPECT(isg_conv_wgrad_rep(&g, nullptr, nullptr, nullptr, nullptr, 0, 4, nullptr) == ISG_ERR_INVALID);
    EXPECT(isg_mask_nms_workspace(16, 1024, 1024) > 0);

    // executor: a malformed record size, an unknown kind, then well-formed records whose
    // launches fail without a device (fix-ups and the side-stream batching run first)
    std::vector<char> blob;
    std::vector<char> big(9000, 0);
    char desc[64] = {};
    put_op(blob, 12, big.data(), (int)big.size(), {}, {});  // larger than the executor's buffer
    void* table[32] = {};
    EXPECT(isg_exec(blob.data(), 1, table, nullptr) == ISG_ERR_INVALID);
    blob.clear();
    put_op(blob, 77, desc, 16, {}, {});
    EXPECT(isg_exec(blob.data(), 1, table, nullptr) == ISG_ERR_INVALID);
    EXPECT(std::strstr(isg_last_error(), "unknown op kind") != nullptr);
    blob.clear();
    std::vector<char> arena(4096);
    table[0] = arena.data();
    struct { void* p; int64_t bytes; } ms{nullptr, 256};
    put_op(blob, 12, &ms, sizeof(ms), {isg_ref{0, 0, 128}}, {0});
    put_op(blob, 12, &ms, sizeof(ms), {isg_ref{0, 0, 0}}, {0}, /*side|fork_now*/ 1 | 4);
    const int rc = isg_exec_ms(blob.data(), 2, table, nullptr, nullptr);
    std::printf("exec of memset records without a device: rc %d (%s)\n", rc, isg_last_error());

    // host item arrays longer than one chunk
    std::vector<isg_bn> bns(3 * ISG_LIST_CHUNK + 5);
    for (auto& b : bns) { std::memset(&b, 0, sizeof(b)); b.C = 16; b.train = 1; b.count = 4.f; b.eps = 1e-5f; }
    const int rb = isg_bn_finalize(bns.data(), (int32_t)bns.size(), 0, nullptr);
    std::vector<isg_bn_update> ups(ISG_LIST_CHUNK + 1);
    std::memset(ups.data(), 0, ups.size() * sizeof(isg_bn_update));
    const int ru = isg_bn_update_running(ups.data(), (int32_t)ups.size(), nullptr);
    std::vector<isg_grad_final> gfs(2 * ISG_LIST_CHUNK);
    std::memset(gfs.data(), 0, gfs.size() * sizeof(isg_grad_final));
    const int rg = isg_grad_finalize(gfs.data(), (int32_t)gfs.size(), nullptr);
    std::printf("chunked item launches without a device: %d %d %d\n", rb, ru, rg);
    EXPECT(isg_bn_finalize(nullptr, 0, 0, nullptr) == ISG_OK || std::strlen(isg_last_error()) > 0);

    std::printf("%s: %d failure(s)\n", failures ? "FAIL" : "OK", failures);
    return failures ? 1 : 0;
}
