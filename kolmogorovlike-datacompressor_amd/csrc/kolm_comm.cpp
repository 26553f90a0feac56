// kolm_comm.cpp — RCCL behind the C ABI: the one exchange step of the multi-GPU path.
//
// Blocks are independent (PY:2350-2369), so ranks encode their block shards with no
// collective; the output stream is reassembled on one rank before the container is written
// (PY:2375-2445).  This file owns that step:
//   * kolm_comm_*            one communicator rank per process (ncclCommInitRank on the
//                            context's device; one process per GPU, xGMI between them);
//   * kolm_gather_payloads   every rank's payload arena, method ids and payload offsets onto
//                            one destination rank's device buffer: a 4-word all-gather of the
//                            per-rank sizes, then ncclSend/ncclRecv of each arena exactly as
//                            long as it is (no padding to the largest rank), placed back to
//                            back in rank order, plus one small packed (offsets, ids) record
//                            per rank; the destination's own part is a device-to-device copy.
//                            Optionally asynchronous (kolm_comm_wait), so the transfer of
//                            batch k runs over xGMI while batch k + 1 encodes;
//   * multi_rccl_gather      kolm_encode_blocks_multi's reassembly: ncclCommInitAll over the
//                            process's devices, every device's payloads received into device
//                            0 in one group, then one copy to the caller's host buffer.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kolm.h"
#include "kolm_internal.h"

using namespace kolm;

static_assert(KOLM_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "kolm.h's id size must match RCCL's");

namespace {

struct RcclError {
    ncclResult_t r;
    const char* what;
    int line;
};
#define KOLM_NCCL_CHECK(x)                                             \
    do {                                                               \
        const ncclResult_t r_ = (x);                                   \
        if (r_ != ncclSuccess) throw RcclError{r_, #x, __LINE__};      \
    } while (0)

template <class F>
int cguard(F&& f) {
    try {
        return f();
    } catch (const RcclError& e) {
        char buf[320];
        snprintf(buf, sizeof buf, "RCCL error %d (%s) at kolm_comm line %d: %s", (int)e.r, ncclGetErrorString(e.r),
                 e.line, e.what);
        set_err(buf);
        return KOLM_ERCCL;
    } catch (const HipError& e) {
        char buf[320];
        snprintf(buf, sizeof buf, "HIP error %d (%s) at kolm_comm line %d: %s", (int)e.err, hipGetErrorString(e.err),
                 e.line, e.what);
        set_err(buf);
        return KOLM_EHIP;
    } catch (const std::bad_alloc&) {
        set_err("host allocation failed");
        return KOLM_EHIP;
    }
}

// grow-only buffers (device / pinned host); contents are not preserved on growth
struct DevMem {
    void* p = nullptr;
    size_t cap = 0;
    template <class T>
    T* get(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (cap < bytes) {
            if (p) KOLM_HIP_CHECK(hipFree(p));
            p = nullptr;
            cap = 0;
            const size_t c = (bytes + 4095) & ~(size_t)4095;
            KOLM_HIP_CHECK(hipMalloc(&p, c));
            cap = c;
        }
        return static_cast<T*>(p);
    }
    void release() noexcept {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};
struct HostMem {
    void* p = nullptr;
    size_t cap = 0;
    template <class T>
    T* get(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (cap < bytes) {
            if (p) KOLM_HIP_CHECK(hipHostFree(p));
            p = nullptr;
            cap = 0;
            const size_t c = (bytes + 4095) & ~(size_t)4095;
            KOLM_HIP_CHECK(hipHostMalloc(&p, c, hipHostMallocDefault));
            cap = c;
        }
        return static_cast<T*>(p);
    }
    void release() noexcept {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// one rank's packed (offsets, ids) record: nblocks + 1 u64 offsets then nblocks u32 ids,
// padded to 8 bytes
inline u64 idx_bytes(u64 nblocks) { return (8 * (nblocks + 1) + 4 * nblocks + 7) & ~7ull; }

// meta words every rank contributes to a gather: sizes, the destination's capacities, the
// destination rank it was called with and whether its own arguments were valid
enum : int { M_BYTES = 0, M_BLOCKS = 1, M_CAP = 2, M_CAPB = 3, M_DST = 4, M_BAD = 5, M_N = 6 };

}  // namespace

struct kolm_comm {
    int device = 0, rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;  // RCCL's stream: the gathers of this communicator
    std::mutex mu;
    DevMem meta_d, idx_send_d, idx_recv_d, red_d;
    HostMem meta_h, idx_send_h, idx_recv_h, red_h;
    // an asynchronous gather in flight on the destination: outputs filled by finish()
    bool pending = false;
    u32* out_method = nullptr;
    u64* out_off = nullptr;
    std::vector<u64> rbytes, pbase;
    std::vector<u32> rblocks;

    // completes the gather in flight (every rank), then unpacks the destination's host outputs
    void finish() {
        if (!pending) return;
        pending = false;
        KOLM_HIP_CHECK(hipStreamSynchronize(stream));
        if (!out_method && !out_off) return;
        const u8* rec = idx_recv_h.get<u8>(0);
        u64 g = 0, ib = 0;
        for (int r = 0; r < nranks; ++r) {
            const u64 nb = rblocks[r];
            const u64* off = reinterpret_cast<const u64*>(rec + ib);
            const u32* ids = reinterpret_cast<const u32*>(rec + ib + 8 * (nb + 1));
            for (u64 i = 0; i < nb; ++i) {
                if (out_method) out_method[g + i] = ids[i];
                if (out_off) out_off[g + i] = pbase[r] + off[i];
            }
            g += nb;
            ib += idx_bytes(nb);
        }
        if (out_off) out_off[g] = pbase[nranks];
        out_method = nullptr;
        out_off = nullptr;
    }
};

namespace {
// kolm_encode_blocks_multi's communicator over this process's devices (ncclCommInitAll)
struct MultiComm {
    std::mutex mu;
    std::vector<int> devs;     // the devices of a complete communicator (empty: none)
    std::vector<int> sdev;     // the device of every communicator / stream slot, set before init
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;
    DevMem dst;  // on sdev[0]
    void reset() noexcept {
        for (size_t i = 0; i < comms.size(); ++i) {
            if (comms[i]) (void)ncclCommDestroy(comms[i]);
            if (i < streams.size() && streams[i]) {
                (void)hipSetDevice(sdev[i]);
                (void)hipStreamDestroy(streams[i]);
            }
        }
        if (!sdev.empty()) {
            (void)hipSetDevice(sdev[0]);
            dst.release();
        }
        comms.clear();
        streams.clear();
        devs.clear();
        sdev.clear();
    }
};
MultiComm g_mc;
}  // namespace

namespace kolm {

// Reassembly of kolm_encode_blocks_multi (kolm_api.cpp): device r holds its shard's payloads
// in d_pay[r][0, nbytes[r]); they are received into device devs[0] back to back (RCCL group:
// one ncclSend per device r > 0 to rank 0, the matching ncclRecv on rank 0; device 0's own
// part by a device-to-device copy) and copied once into host[0, sum).  Returns a KOLM_* code.
int multi_rccl_gather(const std::vector<int>& devs, const std::vector<const u8*>& d_pay,
                      const std::vector<u64>& nbytes, u8* host, u64 cap) {
    return cguard([&] {
        std::lock_guard<std::mutex> g(g_mc.mu);
        const int G = (int)devs.size();
        u64 total = 0;
        std::vector<u64> base(G + 1, 0);
        for (int r = 0; r < G; ++r) base[r + 1] = base[r] + nbytes[r];
        total = base[G];
        if (total > cap) {
            set_err("payload_arena too small");
            return KOLM_ECAP;
        }
        if (g_mc.devs != devs) {
            // the cache records devs only once the communicators and streams all exist: a
            // failure part-way leaves it empty, so the next call initialises again
            g_mc.reset();
            try {
                g_mc.sdev = devs;
                g_mc.comms.assign(G, nullptr);
                g_mc.streams.assign(G, nullptr);
                KOLM_NCCL_CHECK(ncclCommInitAll(g_mc.comms.data(), G, devs.data()));
                for (int r = 0; r < G; ++r) {
                    KOLM_HIP_CHECK(hipSetDevice(devs[r]));
                    KOLM_HIP_CHECK(hipStreamCreateWithFlags(&g_mc.streams[r], hipStreamNonBlocking));
                }
            } catch (...) {
                g_mc.reset();
                throw;
            }
            g_mc.devs = devs;
        }
        if (!total) return KOLM_OK;
        KOLM_HIP_CHECK(hipSetDevice(devs[0]));
        u8* dst = g_mc.dst.get<u8>(total);
        KOLM_NCCL_CHECK(ncclGroupStart());
        for (int r = 1; r < G; ++r) {
            if (!nbytes[r]) continue;
            KOLM_NCCL_CHECK(ncclSend(d_pay[r], nbytes[r], ncclUint8, 0, g_mc.comms[r], g_mc.streams[r]));
            KOLM_NCCL_CHECK(ncclRecv(dst + base[r], nbytes[r], ncclUint8, r, g_mc.comms[0], g_mc.streams[0]));
        }
        KOLM_NCCL_CHECK(ncclGroupEnd());
        KOLM_HIP_CHECK(hipSetDevice(devs[0]));
        if (nbytes[0])
            KOLM_HIP_CHECK(hipMemcpyAsync(dst, d_pay[0], nbytes[0], hipMemcpyDeviceToDevice, g_mc.streams[0]));
        KOLM_HIP_CHECK(hipMemcpyAsync(host, dst, total, hipMemcpyDeviceToHost, g_mc.streams[0]));
        for (int r = 0; r < G; ++r) {
            KOLM_HIP_CHECK(hipSetDevice(devs[r]));
            KOLM_HIP_CHECK(hipStreamSynchronize(g_mc.streams[r]));
        }
        return KOLM_OK;
    });
}

void comm_shutdown() {
    std::lock_guard<std::mutex> g(g_mc.mu);
    g_mc.reset();
}

}  // namespace kolm

extern "C" {

int kolm_comm_unique_id(uint8_t* id) {
    if (!id) return KOLM_EARG;
    return cguard([&] {
        ncclUniqueId u;
        KOLM_NCCL_CHECK(ncclGetUniqueId(&u));
        std::memcpy(id, u.internal, KOLM_COMM_ID_BYTES);
        return KOLM_OK;
    });
}

int kolm_comm_init(kolm_ctx* ctx, int nranks, int rank, const uint8_t* id, kolm_comm** out) {
    // rank / nranks are validated by RCCL itself (ncclInvalidArgument -> KOLM_ERCCL, before
    // any bootstrap traffic)
    if (!ctx || !id || !out) return KOLM_EARG;
    *out = nullptr;
    kolm_comm* c = new (std::nothrow) kolm_comm;
    if (!c) return KOLM_EHIP;
    c->device = ctx_device(ctx);
    c->rank = rank;
    c->nranks = std::max(nranks, 1);
    const int rc = cguard([&] {
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        KOLM_HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        ncclUniqueId u;
        std::memcpy(u.internal, id, KOLM_COMM_ID_BYTES);
        KOLM_NCCL_CHECK(ncclCommInitRank(&c->comm, nranks, u, rank));
        return KOLM_OK;
    });
    if (rc) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
        return rc;
    }
    *out = c;
    return KOLM_OK;
}

int kolm_comm_destroy(kolm_comm* c) {
    if (!c) return KOLM_EARG;
    int rc = cguard([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->finish();
        return KOLM_OK;
    });
    if (c->comm) {
        const ncclResult_t r = ncclCommDestroy(c->comm);
        if (r != ncclSuccess && !rc) {
            set_err(std::string("ncclCommDestroy: ") + ncclGetErrorString(r));
            rc = KOLM_ERCCL;
        }
    }
    (void)hipSetDevice(c->device);
    c->meta_d.release();
    c->idx_send_d.release();
    c->idx_recv_d.release();
    c->red_d.release();
    c->meta_h.release();
    c->idx_send_h.release();
    c->idx_recv_h.release();
    c->red_h.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return rc;
}

int kolm_comm_rank(kolm_comm* c, int* rank, int* nranks) {
    if (!c) return KOLM_EARG;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return KOLM_OK;
}

int kolm_comm_allreduce(kolm_comm* c, void* values, uint32_t count, int dtype, int op) {
    if (!c || (count && !values) || dtype < 0 || dtype > 1 || op < 0 || op > 1) return KOLM_EARG;
    if (!count) return KOLM_OK;
    return cguard([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->finish();
        const size_t bytes = 8ull * count;
        void* h = c->red_h.get<u8>(bytes);
        void* d = c->red_d.get<u8>(bytes);
        std::memcpy(h, values, bytes);
        KOLM_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
        KOLM_NCCL_CHECK(ncclAllReduce(d, d, count, dtype ? ncclFloat64 : ncclUint64, op ? ncclMax : ncclSum, c->comm,
                                      c->stream));
        KOLM_HIP_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->stream));
        std::memcpy(values, h, bytes);
        return KOLM_OK;
    });
}

int kolm_comm_barrier(kolm_comm* c) {
    uint64_t one = 1;
    return kolm_comm_allreduce(c, &one, 1, 0, 0);
}

int kolm_gather_payloads(kolm_comm* c, const void* d_arena, uint64_t nbytes, const uint32_t* method,
                         const uint64_t* payload_off, uint32_t nblocks, int dst, void* d_dst, uint64_t dst_cap,
                         uint32_t dst_cap_blocks, uint64_t* rank_bytes, uint32_t* rank_blocks, uint32_t* method_all,
                         uint64_t* off_all, int async_op) {
    if (!c) return KOLM_EARG;
    // Argument errors are not returned before the collective: a rank that left early would leave
    // the others blocked in it.  Every rank joins the size all-gather with its own verdict and the
    // destination it was given, and all of them return KOLM_EARG together if any rank's
    // arguments are bad or the ranks disagree on the destination.
    const bool dst_ok = dst >= 0 && dst < c->nranks;
    const bool is_dst = dst_ok && c->rank == dst;
    const bool bad = !dst_ok || (nbytes && !d_arena) || (nblocks && (!method || !payload_off)) ||
                     (is_dst && ((!d_dst && dst_cap) || (!method_all && !off_all && dst_cap_blocks)));
    return cguard([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->finish();  // a previous gather still in flight owns the staging buffers
        const int R = c->nranks;
        // (1) per-rank sizes, and the destination's capacities, to every rank
        u64* mh = c->meta_h.get<u64>(8ull * M_N * (R + 1));
        u64* md = c->meta_d.get<u64>(8ull * M_N * (R + 1));
        mh[M_BYTES] = nbytes;
        mh[M_BLOCKS] = nblocks;
        mh[M_CAP] = is_dst ? dst_cap : 0;
        mh[M_CAPB] = is_dst ? dst_cap_blocks : 0;
        mh[M_DST] = (u64)(int64_t)dst;
        mh[M_BAD] = bad ? 1u : 0u;
        KOLM_HIP_CHECK(hipMemcpyAsync(md, mh, 8 * M_N, hipMemcpyHostToDevice, c->stream));
        KOLM_NCCL_CHECK(ncclAllGather(md, md + M_N, M_N, ncclUint64, c->comm, c->stream));
        KOLM_HIP_CHECK(hipMemcpyAsync(mh + M_N, md + M_N, 8ull * M_N * R, hipMemcpyDeviceToHost, c->stream));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->stream));
        const u64* all = mh + M_N;
        for (int r = 0; r < R; ++r)
            if (all[r * M_N + M_BAD] || all[r * M_N + M_DST] != (u64)(int64_t)dst) {
                set_err("kolm_gather_payloads: bad arguments on rank " + std::to_string(r) +
                        " (null buffers, or destination ranks that differ or are out of range)");
                return KOLM_EARG;
            }
        c->rbytes.assign(R, 0);
        c->rblocks.assign(R, 0);
        c->pbase.assign(R + 1, 0);
        u64 tot_blocks = 0, idx_tot = 0;
        std::vector<u64> ibase(R + 1, 0);
        for (int r = 0; r < R; ++r) {
            c->rbytes[r] = all[r * M_N + M_BYTES];
            c->rblocks[r] = (u32)all[r * M_N + M_BLOCKS];
            c->pbase[r + 1] = c->pbase[r] + c->rbytes[r];
            tot_blocks += c->rblocks[r];
            ibase[r + 1] = ibase[r] + idx_bytes(c->rblocks[r]);
        }
        idx_tot = ibase[R];
        if (rank_bytes)
            for (int r = 0; r < R; ++r) rank_bytes[r] = c->rbytes[r];
        if (rank_blocks)
            for (int r = 0; r < R; ++r) rank_blocks[r] = c->rblocks[r];
        // every rank decides the same way: nothing is sent when the destination cannot hold it
        if (c->pbase[R] > all[dst * M_N + M_CAP] || tot_blocks > all[dst * M_N + M_CAPB]) {
            set_err("kolm_gather_payloads: destination capacity too small (rank_bytes / rank_blocks hold the sizes)");
            return KOLM_ECAP;
        }
        // (2) this rank's packed (offsets, ids) record
        const u64 ib = idx_bytes(nblocks);
        u8* sh = c->idx_send_h.get<u8>(ib);
        std::memset(sh, 0, ib);
        if (nblocks) {
            std::memcpy(sh, payload_off, 8ull * (nblocks + 1));
            std::memcpy(sh + 8ull * (nblocks + 1), method, 4ull * nblocks);
        }
        u8* sd = c->idx_send_d.get<u8>(ib);
        KOLM_HIP_CHECK(hipMemcpyAsync(sd, sh, ib, hipMemcpyHostToDevice, c->stream));
        u8* rd = is_dst ? c->idx_recv_d.get<u8>(idx_tot) : nullptr;
        u8* out = static_cast<u8*>(d_dst);
        // (3) arenas and records to the destination, each exactly as long as it is
        KOLM_NCCL_CHECK(ncclGroupStart());
        if (!is_dst) {
            if (nbytes) KOLM_NCCL_CHECK(ncclSend(d_arena, nbytes, ncclUint8, dst, c->comm, c->stream));
            KOLM_NCCL_CHECK(ncclSend(sd, ib, ncclUint8, dst, c->comm, c->stream));
        } else {
            for (int r = 0; r < R; ++r) {
                if (r == dst) continue;
                if (c->rbytes[r])
                    KOLM_NCCL_CHECK(ncclRecv(out + c->pbase[r], c->rbytes[r], ncclUint8, r, c->comm, c->stream));
                KOLM_NCCL_CHECK(ncclRecv(rd + ibase[r], idx_bytes(c->rblocks[r]), ncclUint8, r, c->comm, c->stream));
            }
        }
        KOLM_NCCL_CHECK(ncclGroupEnd());
        if (is_dst) {
            if (nbytes)
                KOLM_HIP_CHECK(
                    hipMemcpyAsync(out + c->pbase[dst], d_arena, nbytes, hipMemcpyDeviceToDevice, c->stream));
            KOLM_HIP_CHECK(hipMemcpyAsync(rd + ibase[dst], sd, ib, hipMemcpyDeviceToDevice, c->stream));
            u8* rh = c->idx_recv_h.get<u8>(idx_tot);
            KOLM_HIP_CHECK(hipMemcpyAsync(rh, rd, idx_tot, hipMemcpyDeviceToHost, c->stream));
            c->out_method = method_all;
            c->out_off = off_all;
        } else {
            c->out_method = nullptr;
            c->out_off = nullptr;
        }
        c->pending = true;
        if (!async_op) c->finish();
        return KOLM_OK;
    });
}

int kolm_comm_wait(kolm_comm* c) {
    if (!c) return KOLM_EARG;
    return cguard([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->finish();
        return KOLM_OK;
    });
}

}  // extern "C"
