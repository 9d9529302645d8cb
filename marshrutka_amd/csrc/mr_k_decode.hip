// mr_k_decode.hip — mr_plan_fetch on the device: the compact records a pass wrote
// (OutResult + command slots / overflow pool, grouped by source) expanded into the ABI's
// mr_result (query order) and mr_command pool, the layout the host decoder writes
// (mr_host.cpp decode_record): query i's commands at the exclusive prefix sum of the
// command counts of queries 0 .. i-1.  The host then copies both arrays once.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../../include/marshrutka_pf.h"
#include "mr_engine.hpp"

namespace mr {

// the record's command count as the pool counts it (0: no commands to write)
__device__ __forceinline__ uint32_t rec_cmds(const OutResult &o) {
    const int st = int(o.ncmd_status >> 16) - 16;
    return (st == MR_OK || st == int(kStatusOverflow)) ? (o.ncmd_status & 0xFFFFu) : 0u;
}

__global__ void decode_count_kernel(const OutResult *__restrict__ res, const uint32_t *__restrict__ q_id, uint32_t nrec,
                                    uint32_t *__restrict__ cnt) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nrec; k += gridDim.x * blockDim.x)
        cnt[q_id[k]] = rec_cmds(res[k]);
}

struct DecodeScale {
    uint32_t rgt, soe, shq, sfm, ff;
};

// one thread per record: its mr_result at its query, its commands at the query's offset
// when they fit pool_cap (else the capacity flag); err bit 0: a malformed record
__global__ void decode_write_kernel(const OutResult *__restrict__ res, const OutCmd *__restrict__ slots,
                                    const OutCmd *__restrict__ ovf, uint32_t novf, const uint32_t *__restrict__ q_id,
                                    uint32_t nrec, uint32_t mc, const uint32_t *__restrict__ off,
                                    const mr_cell_index *__restrict__ idx_rank, uint32_t V, DecodeScale cs,
                                    mr_result *__restrict__ out, mr_command *__restrict__ pool, unsigned long long pool_cap,
                                    uint32_t *__restrict__ err) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nrec; k += gridDim.x * blockDim.x) {
        const OutResult o = res[k];
        const uint32_t q = q_id[k];
        int status = int(o.ncmd_status >> 16) - 16;
        mr_result r;
        r.legs = o.legs;
        r.money = o.money;
        r.time_s = int64_t(o.time);
        r.n_commands = o.ncmd_status & 0xFFFFu;
        r.command_offset = off[q];
        r.reserved = 0;
        const OutCmd *src = slots + (unsigned long long)k * mc;
        if (status == MR_NOT_FOUND) r.n_commands = 0;
        if (status == int(kStatusOverflow)) {  // its commands in the overflow pool at {offset, count}
            const OutCmd tag = src[0];
            if (!mc || tag.kp != kOvfTag || tag.to != r.n_commands || (unsigned long long)tag.from + tag.to > novf) {
                atomicOr(err, 1u);
                r.n_commands = 0;
            }
            src = ovf + tag.from;
            status = MR_OK;
        } else if (status == MR_OK && r.n_commands > mc) {
            atomicOr(err, 1u);
            r.n_commands = 0;  // its slots hold no more than mc commands: read none (decode_record)
        }
        r.status = status;
        out[q] = r;
        if (status != MR_OK) continue;
        if ((unsigned long long)r.command_offset + r.n_commands > pool_cap) {
            atomicOr(err, 2u);
            continue;
        }
        for (uint32_t j = 0; j < r.n_commands; ++j) {
            const OutCmd c = src[j];
            const uint32_t kind = c.kp >> 29, pay = c.kp & 0x1FFFFFFFu;
            mr_command m;
            m.kind = uint8_t(kind);
            m.reserved[0] = m.reserved[1] = m.reserved[2] = 0;
            m.legs = 0;
            m.money = 0;
            m.fleetfoot = 0;
            m.time_s = 0;
            switch (kind) {
                case kCentral: m.time_s = int64_t(10) * pay; break;
                case kStandard:
                    m.legs = pay;
                    m.time_s = int64_t(180) * pay;
                    m.fleetfoot = cs.ff;
                    break;
                case kCaravan:
                    m.time_s = int64_t(cs.rgt) * (pay >> 1);
                    m.money = (pay >> 1) * ((pay & 1u) ? 5u : 2u);
                    break;
                case kSoE: m.money = cs.soe; break;
                case kSHQ: m.money = cs.shq; break;
                case kSFm: m.money = cs.sfm; break;
                default: break;
            }
            if (kind > kSFm || c.from >= V || c.to >= V) {
                atomicOr(err, 1u);
                continue;
            }
            m.from = idx_rank[c.from];  // device commands name cells by rank
            m.to = idx_rank[c.to];
            pool[(unsigned long long)r.command_offset + j] = m;
        }
    }
}

// Device decode of a plan's records into out (n_queries results) and pool; cnt / off
// are n_queries words of scratch (cnt zeroed here), temp scan scratch of *temp_bytes
// (a null temp returns the size needed).  err: one word.
hipError_t decode_records_device(const OutResult *res, const OutCmd *slots, const OutCmd *ovf, uint32_t novf,
                                 const uint32_t *q_id, uint32_t nrec, uint32_t nq, uint32_t mc,
                                 const mr_cell_index *idx_rank, uint32_t V, uint32_t rgt, uint32_t soe, uint32_t shq,
                                 uint32_t sfm, uint32_t ff, uint32_t *cnt, uint32_t *off, void *temp, size_t *temp_bytes,
                                 mr_result *out, mr_command *pool, unsigned long long pool_cap, uint32_t *err,
                                 hipStream_t stream) {
    if (!temp) return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, cnt, off, int(nq), stream);
    hipError_t e = hipMemsetAsync(cnt, 0, size_t(nq) * 4, stream);
    if (e == hipSuccess) e = hipMemsetAsync(err, 0, 4, stream);
    const uint32_t blocks = std::max(1u, std::min(4096u, (nrec + 255) / 256));
    if (e == hipSuccess && nrec)
        hipLaunchKernelGGL(decode_count_kernel, dim3(blocks), dim3(256), 0, stream, res, q_id, nrec, cnt);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, cnt, off, int(nq), stream);
    const DecodeScale cs{rgt, soe, shq, sfm, ff};
    if (e == hipSuccess && nrec)
        hipLaunchKernelGGL(decode_write_kernel, dim3(blocks), dim3(256), 0, stream, res, slots, ovf, novf, q_id, nrec, mc,
                           off, idx_rank, V, cs, out, pool, pool_cap, err);
    if (e == hipSuccess) e = hipGetLastError();
    return e;
}

// ---- wire records (mr_engine.hpp): the records of a pass re-encoded for transfer -------------
// One thread per record: 4 + 8 max_cmds bytes instead of 16 + 16 max_cmds (c4: 36 B a query
// against 80), the metrics left to the decoder; an overflowing label's commands go to the
// wire pool at the same offsets (wpool_cap commands; past it the record reads
// MR_ERR_CAPACITY).  nov: the pass's overflow-pool length, read on the device.
__global__ void wire_kernel(const OutResult *__restrict__ res, const OutCmd *__restrict__ slots,
                            const OutCmd *__restrict__ ovf, const uint32_t *__restrict__ nov_p, uint32_t ovf_cap,
                            uint32_t nrec, uint32_t nq, uint32_t mc, const uint32_t *__restrict__ q_id,
                            const uint32_t *__restrict__ q_off, uint32_t *__restrict__ rows, uint32_t *__restrict__ wpool,
                            uint32_t wpool_cap, bool stage_rows) {
    // (q_off: the fetch's rows, one word longer, ending in the query's offset in the output
    // pool, so that any row decodes on its own)
    const uint32_t nov = min(*nov_p, ovf_cap), rw = 1u + 2u * mc + (q_off ? 1u : 0u);
    // (q_id: rows in query order, record k at row q_id[k]; the rows of queries without a
    // record are left alone)
    const uint32_t nrow = q_id ? nrec : nq;
    // rows in record order are built in LDS (a row per thread; rw odd, so the threads' rows
    // start in distinct banks) and stored by the workgroup as one contiguous run: a thread
    // storing its own 36 B row scatters every store instruction over 36 lines
    extern __shared__ uint32_t wsh[];
    const bool stage = !q_id && stage_rows;
    const uint32_t bd = blockDim.x, tid = threadIdx.x;
    for (uint32_t base = blockIdx.x * bd; base < nrow; base += gridDim.x * bd) {
        const uint32_t k = base + tid;
        if (k >= nrow) {
            if (!stage) continue;
        } else {
            // rows past the records (queries with an invalid cell index) read MR_ERR_INVALID_INDEX
            const OutResult o = k < nrec ? res[k] : OutResult{0u, 0u, 0u, uint32_t(16 + MR_ERR_INVALID_INDEX) << 16};
            const int st = int(o.ncmd_status >> 16) - 16;
            const uint32_t n = o.ncmd_status & 0xFFFFu;
            const OutCmd *src = slots + (unsigned long long)k * mc;
            uint32_t *row = stage ? wsh + tid * rw : rows + (unsigned long long)(q_id ? q_id[k] : k) * rw;
            uint32_t hdr, s0 = 0, s1 = 0;
            bool copy = false;
            if (st == MR_OK && n <= mc && n < kWireOvf) {
                hdr = (n ? (src[0].from & kWireRankMask) : 0u) | (n << kWireRankBits);
                copy = true;
            } else if (st == int(kStatusOverflow) && mc) {
                const OutCmd tag = src[0];
                if (tag.kp == kOvfTag && tag.to == n && (unsigned long long)tag.from + n <= nov &&
                    (unsigned long long)tag.from + n <= wpool_cap && n) {
                    hdr = (ovf[tag.from].from & kWireRankMask) | (kWireOvf << kWireRankBits);
                    s0 = tag.from;
                    s1 = n;
                    for (uint32_t j = 0; j < n; ++j) {
                        const OutCmd c = ovf[tag.from + j];
                        wpool[2ull * (tag.from + j)] = c.kp;
                        wpool[2ull * (tag.from + j) + 1] = c.to;
                    }
                } else {
                    hdr = (kWireStatus + 32u + uint32_t(MR_ERR_CAPACITY)) << kWireRankBits;
                }
            } else {
                hdr = (kWireStatus + 32u + uint32_t(st == MR_OK ? MR_ERR_DEVICE : st)) << kWireRankBits;
            }
            row[0] = hdr;
            for (uint32_t j = 0; j < mc; ++j) {
                uint32_t kp = 0, to = 0;
                if (copy && j < n) {
                    const OutCmd c = src[j];
                    kp = c.kp;
                    to = c.to;
                } else if (j == 0) {
                    kp = s0;
                    to = s1;
                }
                row[1 + 2 * j] = kp;
                row[2 + 2 * j] = to;
            }
            if (q_off) row[1 + 2 * mc] = q_off[q_id ? q_id[k] : k];
        }
        if (stage) {
            __syncthreads();
            const uint32_t nw = min(bd, nrow - base) * rw;
            uint32_t *dst = rows + (unsigned long long)base * rw;
            for (uint32_t w = tid; w < nw; w += bd) dst[w] = wsh[w];
            __syncthreads();
        }
    }
}

hipError_t launch_wire(const OutResult *res, const OutCmd *slots, const OutCmd *ovf, const uint32_t *nov, uint32_t ovf_cap,
                       uint32_t nrec, uint32_t nq, uint32_t mc, const uint32_t *q_id, uint32_t *rows, uint32_t *wpool,
                       uint32_t wpool_cap, hipStream_t stream) {
    const uint32_t nrow = q_id ? nrec : nq;
    if (!nrow) return hipSuccess;
    // (staged rows: 256 threads while their rows fit 64 KB of LDS, else 64, else unstaged)
    const uint32_t rw = 1u + 2u * mc, bd = rw <= 64u ? 256u : 64u;
    const bool stage = !q_id && size_t(bd) * rw * 4 <= 65536;
    const uint32_t blocks = std::max(1u, std::min(8192u, (nrow + bd - 1) / bd));
    hipLaunchKernelGGL(wire_kernel, dim3(blocks), dim3(bd), stage ? size_t(bd) * rw * 4 : 0, stream, res, slots, ovf, nov,
                       ovf_cap, nrec, nq, mc, q_id, nullptr, rows, wpool, wpool_cap, stage);
    return hipGetLastError();
}

// The fetch's wire rows (mr_host.cpp plan_fetch_wire): in query order, each ending in the
// query's command offset (the exclusive prefix of the counts in query order), so the host
// decodes rows in any order on any thread.  cnt / off: nq words of scratch; temp scan
// scratch of *temp_bytes (a null temp returns the size needed).
hipError_t wire_fetch_device(const OutResult *res, const OutCmd *slots, const OutCmd *ovf, const uint32_t *nov,
                             uint32_t ovf_cap, const uint32_t *q_id, uint32_t nrec, uint32_t nq, uint32_t mc, uint32_t *cnt,
                             uint32_t *off, void *temp, size_t *temp_bytes, uint32_t *rows, uint32_t *wpool,
                             uint32_t wpool_cap, hipStream_t stream) {
    if (!temp) return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, cnt, off, int(nq), stream);
    hipError_t e = hipMemsetAsync(cnt, 0, size_t(nq) * 4, stream);
    const uint32_t blocks = std::max(1u, std::min(8192u, (nrec + 255) / 256));
    if (e == hipSuccess && nrec)
        hipLaunchKernelGGL(decode_count_kernel, dim3(blocks), dim3(256), 0, stream, res, q_id, nrec, cnt);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, cnt, off, int(nq), stream);
    if (e == hipSuccess && nrec)
        hipLaunchKernelGGL(wire_kernel, dim3(blocks), dim3(256), 0, stream, res, slots, ovf, nov, ovf_cap, nrec, nq, mc, q_id,
                           off, rows, wpool, wpool_cap, false);
    if (e == hipSuccess) e = hipGetLastError();
    return e;
}

// ---- byte-deterministic overflow pool -----------------------------------
// A pass hands out overflow-pool offsets by atomicAdd, in arrival order, so the raw
// records and the pool differ from run to run in those offsets (the decoded labels do
// not).  For a plan whose raw outputs a collective gathers (mr_plan_bind_outputs_ex with
// an overflow buffer) this one-workgroup kernel runs after the pass: it renumbers the
// offsets as the exclusive prefix sum of the overflowing records' command counts in
// record order, moves each record's commands there through tmp, and publishes the pool's
// new length.  A pass that overflowed nothing costs one load.  (When the pool ran out, the
// records that got no room depend on arrival order: MR_ERR_CAPACITY, not made
// deterministic.)
constexpr uint32_t kOrdBS = 1024;

// record k's overflow segment {from, len} (false: not an overflow record, or a malformed tag)
__device__ __forceinline__ bool ovf_segment(const KArgs *__restrict__ a, uint32_t k, uint32_t nov, uint32_t &from,
                                            uint32_t &len) {
    const OutResult o = a->out_res[k];
    if (int(o.ncmd_status >> 16) - 16 != int(kStatusOverflow)) return false;
    const OutCmd tag = a->out_cmd[(unsigned long long)k * a->p.max_cmds];
    len = o.ncmd_status & 0xFFFFu;
    from = tag.from;
    return tag.kp == kOvfTag && tag.to == len && (unsigned long long)from + len <= nov;
}

__global__ __launch_bounds__(kOrdBS) void ovf_order_kernel(const KArgs *__restrict__ a, uint32_t nrec,
                                                           OutCmd *__restrict__ tmp) {
    __shared__ uint32_t part[kOrdBS];
    uint32_t *c = a->counter;
    const uint32_t nov = min(c[kCtrLastOvf], a->ovf_cap);
    if (nov == 0 || a->p.max_cmds == 0) return;
    const uint32_t t = threadIdx.x;
    const uint32_t lo = uint32_t((unsigned long long)nrec * t / kOrdBS),
                   hi = uint32_t((unsigned long long)nrec * (t + 1) / kOrdBS);
    uint32_t sum = 0;
    for (uint32_t k = lo; k < hi; ++k) {
        uint32_t f, l;
        if (ovf_segment(a, k, nov, f, l)) sum += l;
    }
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < kOrdBS; d <<= 1) {  // inclusive scan of the threads' sums
        const uint32_t v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const uint32_t total = part[kOrdBS - 1];
    uint32_t off = part[t] - sum;
    OutCmd *ovf = a->ovf;
    for (uint32_t k = lo; k < hi; ++k) {  // (each thread rewrites only its own records' tags)
        uint32_t f, l;
        if (!ovf_segment(a, k, nov, f, l)) continue;
        for (uint32_t j = 0; j < l; ++j) tmp[off + j] = ovf[f + j];
        a->out_cmd[(unsigned long long)k * a->p.max_cmds].from = off;
        off += l;
    }
    __threadfence();
    __syncthreads();
    for (uint32_t i = t; i < total; i += kOrdBS) ovf[i] = tmp[i];
    if (t == 0) c[kCtrLastOvf] = total;
}

hipError_t launch_ovf_order(const KArgs *d_args, uint32_t nrec, OutCmd *tmp, hipStream_t stream) {
    hipLaunchKernelGGL(ovf_order_kernel, dim3(1), dim3(kOrdBS), 0, stream, d_args, nrec, tmp);
    return hipGetLastError();
}

}  // namespace mr
