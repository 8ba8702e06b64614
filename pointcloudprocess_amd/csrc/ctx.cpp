// Context, error and memory helpers of the C-ABI (host code, built by hipcc).
#include <cstdarg>
#include <csignal>
#include <cstdio>
#include <dlfcn.h>
#include <execinfo.h>
#include <ucontext.h>
#include <unistd.h>
#include <algorithm>
#include <cstring>
#include <iterator>

#include "common.hpp"

namespace pcp {

int set_error(pcp_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        ctx->last_error = buf;
    }
    return code;
}

int hip_fail(pcp_ctx* ctx, hipError_t e, const char* what, const char* file, int line) {
    (void)hipGetLastError();
    return set_error(ctx, e == hipErrorOutOfMemory ? PCP_ERR_NOMEM : PCP_ERR_HIP,
                     "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
}

int scratch(pcp_ctx* ctx, size_t bytes, void** out) {
    if (bytes > ctx->scratch_bytes) {
        if (ctx->scratch) {
            PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
            PCP_HIP(ctx, hipFree(ctx->scratch));
            ctx->scratch = nullptr;
            ctx->scratch_bytes = 0;
        }
        size_t want = bytes + bytes / 4 + 4096;
        hipError_t e = hipMalloc(&ctx->scratch, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return set_error(ctx, PCP_ERR_NOMEM, "scratch hipMalloc(%zu) failed", want);
        }
        ctx->scratch_bytes = want;
    }
    *out = ctx->scratch;
    return PCP_OK;
}

static size_t round_block(size_t b) {
    const size_t g = b >= ((size_t)1 << 20) ? ((size_t)2 << 20) : 4096;
    return (b + g - 1) / g * g;
}

int cache_alloc(pcp_ctx* ctx, size_t bytes, void** p) {
    *p = nullptr;
    const size_t want = round_block(bytes ? bytes : 1);
    auto it = ctx->free_blocks.lower_bound(want);
    if (it != ctx->free_blocks.end() && it->first <= want + want / 4 + ((size_t)2 << 20)) {
        *p = it->second;
        ctx->cached_bytes -= it->first;
        ctx->free_blocks.erase(it);
        return PCP_OK;
    }
    hipError_t e = hipMalloc(p, want);
    if (e != hipSuccess && !ctx->free_blocks.empty()) {  // give the cache back and retry
        (void)hipGetLastError();
        cache_release(ctx);
        e = hipMalloc(p, want);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return set_error(ctx, PCP_ERR_NOMEM, "hipMalloc(%zu bytes) failed: %s", want, hipGetErrorString(e));
    }
    ctx->block_size[*p] = want;
    return PCP_OK;
}

void dfree(pcp_ctx* ctx, void* p) {
    if (!p) return;
    auto it = ctx ? ctx->block_size.find(p) : decltype(ctx->block_size.end()){};
    if (!ctx || it == ctx->block_size.end()) {
        (void)hipFree(p);
        return;
    }
    if (ctx->closing) {  // nothing is cached on a closing context
        ctx->block_size.erase(it);
        (void)hipFree(p);
        return;
    }
    ctx->free_blocks.emplace(it->second, p);
    ctx->cached_bytes += it->second;
    // over the cap: drop the largest cached blocks (stream work using them is complete
    // before hipFree returns, hipFree synchronises)
    while (ctx->cached_bytes > ctx->cache_cap && !ctx->free_blocks.empty()) {
        auto last = std::prev(ctx->free_blocks.end());
        ctx->cached_bytes -= last->first;
        ctx->block_size.erase(last->second);
        (void)hipFree(last->second);
        ctx->free_blocks.erase(last);
    }
}

hipError_t event_get(pcp_ctx* ctx, hipEvent_t* ev) {
    if (!ctx->event_pool.empty()) {
        *ev = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return hipSuccess;
    }
    return hipEventCreate(ev);
}

void event_put(pcp_ctx* ctx, hipEvent_t ev) {
    if (ev) ctx->event_pool.push_back(ev);
}

void cache_release(pcp_ctx* ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->free_blocks) {
        ctx->block_size.erase(kv.second);
        (void)hipFree(kv.second);
    }
    ctx->free_blocks.clear();
    ctx->cached_bytes = 0;
}

// the rest of pcp_ctx_destroy, once no object uses the context any more
static void ctx_finish(pcp_ctx* ctx) {
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->block_size) (void)hipFree(kv.first);  // (blocks an object leaked)
    ctx->block_size.clear();
    for (hipEvent_t ev : ctx->event_pool) (void)hipEventDestroy(ev);
    ctx->event_pool.clear();
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int side_stream(pcp_ctx* ctx, hipStream_t* out) {
    if (!ctx->side) PCP_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    *out = ctx->side;
    return PCP_OK;
}

void ctx_retain(pcp_ctx* ctx) {
    if (ctx) ctx->live++;
}

void ctx_release(pcp_ctx* ctx) {
    if (!ctx) return;
    if (--ctx->live == 0 && ctx->closing) ctx_finish(ctx);
}

}  // namespace pcp

extern "C" {

int pcp_abi_version(void) { return PCP_ABI_VERSION; }

int pcp_ctx_create(int device, void* stream, pcp_ctx** out) {
    if (!out) return PCP_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return PCP_ERR_HIP;
    }
    if (device < 0 || device >= ndev) return PCP_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return PCP_ERR_HIP;
    pcp_ctx* c = new pcp_ctx();
    c->device = device;
    c->stream = (hipStream_t)stream;  // NULL = the device's default (null) stream
    size_t fr = 0, tot = 0;
    // scratch cache: up to a third of HBM, so a pipeline's largest temporaries (C5's sorted-order
    // rows at 200M points are ~52 GB) are reused across calls instead of freed and re-mapped;
    // cache_alloc gives the cache back and retries when an allocation fails
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) c->cache_cap = tot / 3;
    *out = c;
    return PCP_OK;
}

int pcp_ctx_destroy(pcp_ctx* ctx) {
    if (!ctx || ctx->closing) return PCP_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->scan_status) (void)hipFree(ctx->scan_status);
    ctx->scratch = nullptr;
    ctx->scan_status = nullptr;
    pcp::cache_release(ctx);
    ctx->closing = true;
    if (ctx->live == 0) pcp::ctx_finish(ctx);  // else the last object's destroy finishes it
    return PCP_OK;
}

int pcp_ctx_set_stream(pcp_ctx* ctx, void* stream) {
    if (!ctx) return PCP_ERR_ARG;
    if (ctx->own_stream) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
        ctx->own_stream = false;
    }
    ctx->stream = (hipStream_t)stream;
    return PCP_OK;
}

void* pcp_ctx_stream(pcp_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

const char* pcp_last_error(const pcp_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null ctx"; }

int pcp_sync(pcp_ctx* ctx) {
    if (!ctx) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

int pcp_malloc(pcp_ctx* ctx, void** p, size_t bytes) {  // caller memory: not cached
    if (!ctx || !p) return PCP_ERR_ARG;
    hipError_t e = hipMalloc(p, bytes ? bytes : 1);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return pcp::set_error(ctx, PCP_ERR_NOMEM, "hipMalloc(%zu bytes) failed", bytes);
    }
    return PCP_OK;
}

int pcp_free(pcp_ctx* ctx, void* p) {
    if (!ctx) return PCP_ERR_ARG;
    if (p) PCP_HIP(ctx, hipFree(p));
    return PCP_OK;
}

int pcp_memcpy_h2d(pcp_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return PCP_ERR_ARG;
    if (bytes) PCP_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

int pcp_memcpy_d2h(pcp_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return PCP_ERR_ARG;
    if (bytes) PCP_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

int pcp_memset(pcp_ctx* ctx, void* dst, int value, size_t bytes) {
    if (!ctx || (bytes && !dst)) return PCP_ERR_ARG;
    if (bytes) PCP_HIP(ctx, hipMemsetAsync(dst, value, bytes, ctx->stream));
    return PCP_OK;
}

}  // extern "C"

// ---- fault report: name the library (dladdr) and the native frames of a fatal signal, then
// hand the signal to whatever handler was installed before (Python's faulthandler prints the
// Python stack) or to the default action.  Diagnostics only; nothing here runs on a good path.
namespace {
constexpr int kFaultSigs[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
struct sigaction g_prev[sizeof(kFaultSigs) / sizeof(kFaultSigs[0])];
bool g_fault_installed = false;

void fault_write(const char* s) { (void)!write(2, s, std::strlen(s)); }

// async-signal-safe formatting (no snprintf in the handler): decimal and hex into a caller
// buffer, each clamped to `end` like fault_str (a long symbol name may fill the buffer)
char* fault_dec(char* p, unsigned long v, const char* end) {
    char t[24];
    int n = 0;
    do { t[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (n && p < end) *p++ = t[--n];
    return p;
}
char* fault_hex(char* p, unsigned long v, const char* end) {
    char t[20];
    int n = 0;
    do { t[n++] = "0123456789abcdef"[v & 15]; v >>= 4; } while (v);
    t[n++] = 'x';
    t[n++] = '0';
    while (n && p < end) *p++ = t[--n];
    return p;
}
char* fault_str(char* p, const char* s, const char* end) {
    while (*s && p < end) *p++ = *s++;
    return p;
}

void fault_handler(int sig, siginfo_t* si, void* ucv) {
    char buf[1024];
    const char* const end = buf + sizeof(buf) - 2;
    void* pc = nullptr;
#if defined(__x86_64__)
    pc = (void*)((ucontext_t*)ucv)->uc_mcontext.gregs[REG_RIP];
#endif
    // dladdr reads the loader's already-built link map (no allocation on glibc); best effort
    Dl_info di{};
    const bool named = pc && dladdr(pc, &di) && di.dli_fname;
    char* p = fault_str(buf, "[pcp fault] signal ", end);
    p = fault_dec(p, (unsigned long)sig, end);
    p = fault_str(p, " at address ", end);
    p = fault_hex(p, (unsigned long)(si ? si->si_addr : nullptr), end);
    p = fault_str(p, ", pc ", end);
    p = fault_hex(p, (unsigned long)pc, end);
    p = fault_str(p, " in ", end);
    p = fault_str(p, named ? di.dli_fname : "?", end);
    p = fault_str(p, " (", end);
    p = fault_str(p, named && di.dli_sname ? di.dli_sname : "?", end);
    p = fault_str(p, "+", end);
    p = fault_hex(p, named ? (unsigned long)((char*)pc - (char*)(di.dli_sname ? di.dli_saddr : di.dli_fbase)) : 0ul, end);
    p = fault_str(p, ")", end);
    *p++ = '\n';  // end leaves room for it
    (void)!write(2, buf, (size_t)(p - buf));
    void* frames[48];
    const int n = backtrace(frames, 48);
    backtrace_symbols_fd(frames, n, 2);
    // chain: the previous handler, else the default action
    for (size_t k = 0; k < sizeof(kFaultSigs) / sizeof(kFaultSigs[0]); k++) {
        if (kFaultSigs[k] != sig) continue;
        sigaction(sig, &g_prev[k], nullptr);
        const struct sigaction& pv = g_prev[k];
        if ((pv.sa_flags & SA_SIGINFO) && pv.sa_sigaction) {
            pv.sa_sigaction(sig, si, ucv);
            return;
        }
        if (pv.sa_handler != SIG_DFL && pv.sa_handler != SIG_IGN && pv.sa_handler) {
            pv.sa_handler(sig);
            return;
        }
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
}  // namespace

extern "C" int pcp_fault_report_install(void) {
    if (g_fault_installed) return PCP_OK;
    // backtrace() loads libgcc's unwinder (malloc, dlopen) on its first call: do that here, not
    // inside a handler that may have interrupted malloc
    void* warm[2];
    (void)backtrace(warm, 2);
    // an alternate stack for this thread, so a stack overflow still reaches the report (kept
    // if one is already installed, e.g. by Python's faulthandler)
    stack_t cur{};
    if (sigaltstack(nullptr, &cur) == 0 && (cur.ss_flags & SS_DISABLE)) {
        static char alt[64 * 1024];
        stack_t ss{};
        ss.ss_sp = alt;
        ss.ss_size = sizeof(alt);
        (void)sigaltstack(&ss, nullptr);
    }
    for (size_t k = 0; k < sizeof(kFaultSigs) / sizeof(kFaultSigs[0]); k++) {
        struct sigaction sa{};
        sa.sa_sigaction = fault_handler;
        sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigemptyset(&sa.sa_mask);
        if (sigaction(kFaultSigs[k], &sa, &g_prev[k]) != 0) return PCP_ERR_ARG;
    }
    g_fault_installed = true;
    return PCP_OK;
}
