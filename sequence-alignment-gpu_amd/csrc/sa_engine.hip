// MI355X (gfx950 / CDNA4) alignment engine, host side and small kernels: the C ABI of sa_hip.h
// (plans, the one-shot sa_align_pair, the per-device workspace), text encoding and the self-test.
//
// Replaces the reference's GPU path (robertszafa/sequence-alignment-gpu alignSequenceGPU.cu:73-653)
// with a new design; see DESIGN.md and sa_layout.h for the data layout. Semantics follow the
// reference CPU path (alignSequenceCPU.cpp), bit-exact:
//   cell recurrence and tie rule      alignSequenceCPU.cpp:175-190 (local), :259-273 (global)
//   boundaries                        :145-149, :163-164 (local), :232-236, :247-248 (global)
//   local best cell (first max)       :191-192
//   tracebacks                        traceBackNW :64-114, traceBackSW :10-62
// Kernels: the DP fill (sa_fill.hip, one translation unit per strip height), the traceback walk
// and expansion (sa_walk.hip), and encode_text_kernel / selftest_kernel here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include "sa_fill.h"
#include "sa_hip.h"
#include "sa_layout.h"
#include "sa_walk.h"
#include "sa_wave.h"

namespace sa {

// Text codes for the fill (layout per score kind, see ScoreKind):
//   kProf / kTable  one dword per letter, 8*c (packed-profile bit offset) or c (LDS table index);
//   kArr            A dword arrays of code_len: array a holds table[a][t[x]] at kPad + x;
//   kArr8           4A byte arrays of code_len bytes: copy (a, r) holds table[a][t[x]] at kPad + x + r.
__global__ void encode_text_kernel(const int8_t *text, const int8_t *pattern, const PairDesc *pairs, int32_t *codes,
                                   int A, int SK, const int32_t *table, Control *ctrl, uint32_t epoch)
{
    // the fill's control word starts here (no memset launch before each fill): the queues and the
    // abort flag at zero; bad_input carries the epoch of the fill it reports, so it needs no reset
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    {
        ctrl->queue_head = 0;
        ctrl->band_head = 0;
        ctrl->abort_flag = 0;
    }
    const PairDesc pd = pairs[blockIdx.y];
    // the arenas must hold alphabet indices 0..A-1 (Request::textBytes / patternBytes are indices,
    // utilities.cpp:52); the kernels clamp, so a bad byte is reported instead of aligned silently
    bool bad = false;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < pd.pattern_len;
         x += (uint64_t)gridDim.x * blockDim.x)
    {
        const int c = pattern[pd.pattern_off + x];
        bad = bad || c < 0 || c >= A;
    }
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < pd.text_len;
         x += (uint64_t)gridDim.x * blockDim.x)
    {
        const int c = text[pd.text_off + x];
        bad = bad || c < 0 || c >= A;
    }
    if (bad) __hip_atomic_store(&ctrl->bad_input, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (SK == kPair)
    {
        // selectors of pairs (2q, 2q+1) in pair 2q's block, padding included (0x0c0c0c0c = zeros)
        if ((blockIdx.y & 1) != 0) return;
        // the column profile of each letter t (byte r = S[r][t] + 2g; A <= 4) from LDS, both pairs'
        // columns in one 8-byte store
        __shared__ uint32_t prof[4];
        if (threadIdx.x < (unsigned)A)
        {
            uint32_t c = 0;
            for (int r = 0; r < A; ++r) c |= ((uint32_t)table[r * A + threadIdx.x] & 0xffu) << (8 * r);
            prof[threadIdx.x] = c;
        }
        __syncthreads();
        const PairDesc pb = pairs[blockIdx.y + 1];
        uint2 *col = reinterpret_cast<uint2 *>(codes + pd.code_off);
        for (uint64_t xx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; xx < pd.code_len;
             xx += (uint64_t)gridDim.x * blockDim.x)
        {
            const int64_t x = (int64_t)xx - kPad;
            uint2 v = {0u, 0u};  // padding: zero scores
            if (x >= 0 && x < (int64_t)pd.text_len)
            {
                v.x = prof[min(max((int)text[pd.text_off + x], 0), A - 1)];
                v.y = prof[min(max((int)text[pb.text_off + x], 0), A - 1)];
            }
            col[xx] = v;
        }
        return;
    }
    // every position of the code block, padding included (zero scores / letter 0): the block is not
    // cleared beforehand
    const int64_t n = (int64_t)pd.text_len;
    auto letter = [&](int64_t x) { return min(max((int)text[pd.text_off + x], 0), A - 1); };
    if (SK == kArr8)
    {
        // copy sh of row r holds S[r][t[p - kPad - sh]] at byte p. One item = (dword w, row r): the
        // four copies' dwords at bytes 4w .. 4w+3, from the 7 letters x0-3 .. x0+3 (x0 = 4w - kPad)
        // and the score table staged in LDS
        __shared__ int8_t tab[32 * 32];
        for (int e = threadIdx.x; e < A * A; e += blockDim.x) tab[e] = (int8_t)table[e];
        __syncthreads();
        uint32_t *w32 = reinterpret_cast<uint32_t *>(codes + pd.code_off);
        const uint64_t rowW = pd.code_len / 4;  // dwords per row (code_len is a multiple of 4)
        const uint64_t items = rowW * (uint64_t)A;
        for (uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items; it += (uint64_t)gridDim.x * blockDim.x)
        {
            const uint64_t w = it % rowW;
            const int r = (int)(it / rowW);
            const int64_t x0 = 4 * (int64_t)w - kPad;
            uint32_t sc[7];  // score byte of each letter (0 outside the text)
            for (int k = 0; k < 7; ++k)
            {
                const int64_t x = x0 - 3 + k;
                sc[k] = (x >= 0 && x < n) ? (uint32_t)(uint8_t)tab[r * A + letter(x)] : 0u;
            }
            for (int sh = 0; sh < 4; ++sh)
                w32[((uint64_t)r * 4 + sh) * rowW + w] =
                    sc[3 - sh] | (sc[4 - sh] << 8) | (sc[5 - sh] << 16) | (sc[6 - sh] << 24);
        }
        return;
    }
    for (uint64_t pp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; pp < pd.code_len;
         pp += (uint64_t)gridDim.x * blockDim.x)
    {
        const int64_t x = (int64_t)pp - kPad;
        if (SK == kArr)
        {
            const int c = (x >= 0 && x < n) ? letter(x) : -1;
            for (int r = 0; r < A; ++r) codes[pd.code_off + (uint64_t)r * pd.code_len + pp] = c >= 0 ? table[r * A + c] : 0;
        }
        else
        {
            const int c = (x >= 0 && x < n) ? letter(x) : 0;
            codes[pd.code_off + pp] = SK == kProf ? 8 * c : c;
        }
    }
}
// ------------------------------------------------------------------------------------------------
// self test of the wave primitives the kernels rely on
// ------------------------------------------------------------------------------------------------
__global__ void selftest_kernel(int *out)
{
    const int lane = threadIdx.x;
    const int v = 100 + lane;
    out[0 * 64 + lane] = dpp_shr1(-1, v);   // expect lane-1 (lane 0: -1)
    out[1 * 64 + lane] = dpp_shl1(-2, v);   // expect lane+1 (lane 63: -2)
    out[2 * 64 + lane] = dpp_rol1(v);       // expect lane+1 mod 64
    const uint64_t b = ballot((lane % 3) == 0);
    uint32_t acc = 0;
    writelane<5>(acc, (uint32_t)b);
    writelane<6>(acc, (uint32_t)(b >> 32));
    out[3 * 64 + lane] = (int)acc;
    out[4 * 64 + lane] = __builtin_amdgcn_sbfe(0x18F70A05, 8 * (lane & 3), 8);  // 5, 10, -9, 24
    // constant 100 MHz clock used by the hand-off timeout must advance
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 2000; ++k) __builtin_amdgcn_s_sleep(10);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[5 * 64 + lane] = (int)(t1 - t0);
}

}  // namespace sa

// ==================================================================================================
// host side
// ==================================================================================================
using namespace sa;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

}  // namespace

namespace sa {
int set_error(int code, const std::string &msg) { return fail(code, msg); }
}  // namespace sa

namespace {

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(SA_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// Environment knobs, read once per process (the first time the engine needs one) and never again:
// every field is a tuning or debugging switch; the defaults are the measured best settings.
struct Knobs {
    bool debug_sync = false;        // SA_DEBUG_SYNC: synchronise and check after every launch
    int rows_per_lane = 0;          // SA_ROWS_PER_LANE: force R (1..32)
    int waves_per_group = 0;        // SA_WAVES_PER_GROUP: force W (1..4)
    bool no_pair16 = false;         // SA_NO_PAIR16: disable the pair-packed batch fill
    int band = -1;                  // SA_BAND: 1 / 0 force the band fill (128-row score strips
                                    // feeding the 64-row strips, sa_fill.hip process_band) on / off
                                    // (1 also past kBandPersistRows*); default: on wherever it applies
                                    // (plan_create)
    double handoff_timeout_s = 20;  // SA_HANDOFF_TIMEOUT_S: in-kernel hand-off give-up time
    int io_sleep = 4;               // SA_IO_SLEEP: I/O wave idle poll period (s_sleep units)
    int chain_lds_kb = 0;           // SA_CHAIN_LDS_KB: dynamic LDS per chain workgroup
    const char *timeline = nullptr; // SA_TIMELINE=<file>: per-strip fill timestamps
    const char *tb_timing = nullptr;// SA_TB_TIMING=<file>: per-pair traceback timestamps
    const char *tb_table_timing = nullptr;  // SA_TB_TABLE_TIMING=<file>: per-strip table kernel stamps
    bool tb_generic = false;        // SA_TB_GENERIC: row walk without the unrolled strip code
    bool tb_stager = true;          // SA_TB_STAGER=0: the row walker stages every strip itself
    bool tb_tables = true;          // SA_TB_TABLES=0: no table traceback (every pair walks sequentially)
    int tb_rounds = 0;              // SA_TB_ROUNDS: rounds of tables (default: plan_traceback)
    bool tb_strict = false;         // SA_TB_STRICT: no sequential walk after the table traceback
                                    // (tests: a pair it left keeps a stale head and fails its check)
    int max_cus = 0;                // SA_MAX_CUS: plan as if the device had at most this many CUs (tests)
    int chain_per_cu = 0;           // SA_CHAIN_PER_CU: 1 / 2 chain workgroups per CU (default: plan_create)
    int64_t band_rows = 0;          // SA_BAND_ROWS: band fill up to this many rows past resident
                                    // capacity (default kBandPersistRows*)
    int pair_chain_r = 0;           // SA_PAIR_CHAIN_R: rows per lane of small batches' pair-packed chains (4 / 8)
    int tb_cap = 0;                 // SA_TB_CAP: column-walk waves at most (0: one per pair)
    bool tb_wide = true;            // SA_TB_WIDE=0: strip tables always 512 threads per strip
    bool stage_kernel = true;       // SA_STAGE_KERNEL=0: one-shot calls stage through DMA copies
    int align = 1;                  // SA_ALIGN=0: chains of alphabets larger than 4 read the four
                                    // byte copies of their text profiles (kArr8) instead of copy 0
                                    // shifted in registers (kArr8A); 2: every alphabet (experiments)
};

const Knobs &knobs()
{
    static const Knobs k = [] {
        Knobs v;
        auto get = [](const char *name) -> const char * { return std::getenv(name); };
        v.debug_sync = get("SA_DEBUG_SYNC") != nullptr;
        if (const char *e = get("SA_ROWS_PER_LANE")) v.rows_per_lane = std::atoi(e);
        if (const char *e = get("SA_WAVES_PER_GROUP")) v.waves_per_group = std::atoi(e);
        v.no_pair16 = get("SA_NO_PAIR16") != nullptr;
        if (const char *e = get("SA_BAND")) v.band = std::atoi(e) != 0 ? 1 : 0;
        if (const char *e = get("SA_HANDOFF_TIMEOUT_S")) v.handoff_timeout_s = std::atof(e);
        if (const char *e = get("SA_IO_SLEEP")) v.io_sleep = std::max(0, std::atoi(e));
        if (const char *e = get("SA_CHAIN_LDS_KB")) v.chain_lds_kb = std::max(0, std::atoi(e));
        v.timeline = get("SA_TIMELINE");
        v.tb_timing = get("SA_TB_TIMING");
        v.tb_table_timing = get("SA_TB_TABLE_TIMING");
        v.tb_generic = get("SA_TB_GENERIC") != nullptr;
        if (const char *e = get("SA_TB_STAGER")) v.tb_stager = std::atoi(e) != 0;
        if (const char *e = get("SA_TB_TABLES")) v.tb_tables = std::atoi(e) != 0;
        v.tb_strict = get("SA_TB_STRICT") != nullptr;
        if (const char *e = get("SA_TB_ROUNDS")) v.tb_rounds = std::max(0, std::atoi(e));
        if (const char *e = get("SA_MAX_CUS")) v.max_cus = std::max(0, std::atoi(e));
        if (const char *e = get("SA_CHAIN_PER_CU")) v.chain_per_cu = std::min(2, std::max(0, std::atoi(e)));
        if (const char *e = get("SA_BAND_ROWS")) v.band_rows = std::max(0LL, std::atoll(e));
        if (const char *e = get("SA_PAIR_CHAIN_R")) v.pair_chain_r = std::atoi(e) == 4 ? 4 : 8;
        if (const char *e = get("SA_TB_CAP")) v.tb_cap = std::max(0, std::atoi(e));
        if (const char *e = get("SA_TB_WIDE")) v.tb_wide = std::atoi(e) != 0;
        if (const char *e = get("SA_STAGE_KERNEL")) v.stage_kernel = std::atoi(e) != 0;
        if (const char *e = get("SA_ALIGN")) v.align = std::min(2, std::max(0, std::atoi(e)));
        return v;
    }();
    return k;
}

// SA_DEBUG_SYNC=1: synchronise and check after every launch (names the failing kernel).
// Makes `device` current for a scope and restores the caller's device on every return path.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int device)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(device) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// Device buffer released on every return path (debug dumps).
struct DevFree {
    void operator()(void *p) const { (void)hipFree(p); }
};
template <typename T>
using DevPtr = std::unique_ptr<T, DevFree>;

int debug_sync(hipStream_t st, const char *what)
{
    if (!knobs().debug_sync) return SA_OK;
    hipError_t e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    std::fprintf(stderr, "[sa debug] %s ok\n", what);
    return SA_OK;
}

template <typename T>
int dmalloc(T **p, size_t bytes)
{
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    if (hipMalloc((void **)p, bytes) != hipSuccess)
    {
        (void)hipGetLastError();
        *p = nullptr;
        return fail(SA_ERR_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes failed");
    }
    return SA_OK;
}

}  // namespace

struct sa_plan {
    int device = 0;
    int mode = 0, A = 0, gap = 0, R = 0, U = 0, W = 1, key_bits = 12, key_rowbits = 21;
    int sk = 0;          // ScoreKind of the fill
    bool chain = false;  // some pair has more than one strip
    bool chain_solo = false;  // one chain workgroup per CU (one compute wave per SIMD), see plan_create
    // band fill (R = 1 int8-profile chains): 128-row score strips ahead of the 64-row strips
    bool band = false;
    std::vector<StripDesc> bands;
    StripDesc *d_bands = nullptr;
    int num_cu = 0;
    std::vector<PairDesc> pairs;
    std::vector<StripDesc> strips;
    char alphabet[33] = {0};
    uint32_t epoch = 0;
    uint32_t *epoch_src = nullptr;  // workspace plans draw epochs from their DeviceCtx (see there)
    hipStream_t own = nullptr;
    // device
    PairDesc *d_pairs = nullptr;
    StripDesc *d_strips = nullptr;
    int32_t *d_prof = nullptr, *d_table = nullptr;
    int32_t *d_codes = nullptr;
    uint32_t *d_masks = nullptr;
    uint64_t *d_bnd = nullptr, *d_best = nullptr;
    int32_t *d_score = nullptr;
    Control *d_ctrl = nullptr;
    int32_t *d_rec = nullptr;  // traceback records (sa_walk.h)
    TbHead *d_heads = nullptr;
    // table traceback (sa_walk.h TbArgs; R = 1 plans with a pair of kTbMinStrips strips or more)
    std::vector<TbGroup> tb_groups;
    std::vector<int32_t> tb_pg;  // [np + 1] first group of each pair
    int64_t tb_slots = 0;        // strip tables (the strips of pairs with groups)
    TbGroup *d_tbgroups = nullptr;
    int32_t *d_tbpg = nullptr, *d_tbl = nullptr, *d_gtbl = nullptr, *d_gent = nullptr, *d_tbflag = nullptr, *d_win = nullptr;
    int32_t *d_tbstart = nullptr, *d_sent = nullptr, *d_sdelta = nullptr, *d_send = nullptr, *d_pend = nullptr;
    int64_t *d_csum = nullptr;  // expansion: per-chunk sums (pairs of more than kChunkRecs records)
    uint64_t *d_cflag = nullptr;  // expansion: per-chunk epoch flags (ExpandArgs::chunk_flags)
    int64_t max_recs = 1;       // records per pair at most (row walk: pattern rows, column walk: text columns)
    char *d_out_text = nullptr, *d_out_pattern = nullptr;
    sa_result *d_results = nullptr;
    const int8_t *d_text_in = nullptr, *d_pattern_in = nullptr;
    uint64_t bytes_total = 0, bytes_masks = 0, out_bytes = 0;
    bool filled = false;
    bool borrowed = false;  // device buffers and stream belong to a DeviceCtx workspace (sa_align_pair)
    // workspace plans: the uploaded region [pairs .. inputs .. ctrl] and the downloaded region
    // [ctrl | results | out_text | out_pattern] are contiguous in the arena (one copy each way)
    char *d_up = nullptr, *d_dn = nullptr;
    size_t up_bytes = 0, dn_bytes = 0;
    int8_t *d_ws_text = nullptr, *d_ws_pattern = nullptr;
    bool ctrl_ready = false;  // the control word was uploaded zeroed (no memset before the next fill)
    std::vector<int32_t> h_prof, h_table;  // host copies the (asynchronous) uploads read from
};

namespace {

// Whether the pairs can run pair-packed (fill_pair_kernel / fill_pair_chain_kernel), whatever R:
// global, an even number of pairs of one shape, a DNA-sized alphabet, every S + 2g in [0, 255] and
// every shifted-domain value within u16 (65534 at most: chains mark unpublished LDS entries with
// 0xffffffff, see sa_fill.hip)
bool pair_packable(const sa_params *P, const sa_pair *pairs, int64_t np)
{
    const int A = P->alphabet_size;
    const int64_t g = P->gap_penalty;
    if (P->mode != SA_GLOBAL || np < 2 || np % 2 != 0 || A > 4 || g <= 0 || knobs().no_pair16) return false;
    int64_t smaxp = 0;
    for (int e = 0; e < A * A; ++e)
    {
        const int64_t v = P->score_matrix[e] + 2 * g;
        if (v < 0 || v > 255) return false;
        smaxp = std::max(smaxp, v);
    }
    for (int64_t p = 0; p < np; ++p)
        if (pairs[p].text_len != pairs[0].text_len || pairs[p].pattern_len != pairs[0].pattern_len)
            return false;
    const uint64_t n = pairs[0].text_len, m = pairs[0].pattern_len;
    return n > 0 && m > 0 && (uint64_t)smaxp * std::min(n, m) <= 65534;
}

int choose_R(const sa_params *P, const sa_pair *pairs, int64_t np, int num_cu)
{
    int R = P->rows_per_lane;
    if (knobs().rows_per_lane) R = knobs().rows_per_lane;
    if (R == 1 || R == 2 || R == 4 || R == 8 || R == 16 || R == 32) return R;
    uint64_t mmax = 0;
    for (int64_t p = 0; p < np; ++p) mmax = std::max<uint64_t>(mmax, pairs[p].pattern_len);
    if (np >= 256)
    {
        // many independent pairs: one strip per pair where possible (no hand-offs at all); local
        // mode keeps 3 registers per row (H, G, best key) and stops at 16 rows per lane, where
        // its working set still fits the register file
        const int rmax = P->mode == SA_LOCAL ? 16 : 32;
        int r = 1;
        while (r < rmax && (uint64_t)kWave * r < mmax) r <<= 1;
        if (pair_packable(P, pairs, np))
        {
            // size the plan to the GPU: a couple of pairs is one wave per strip, and a batch with
            // fewer waves than SIMDs (a shard of the batch on one of N GPUs) leaves SIMDs idle, its
            // time set by one wave's n + 64 steps of R rows. Strips of 8 rows per lane chained in LDS
            // (fill_pair_chain_kernel) split each couple over up to kPairChainMax waves. Measured on
            // config 5's shards (profiles/r06/shard_sweep_v1.log): 1024 pairs 0.86 ms at R = 8 against
            // 1.22 at 16 and 1.24 at 32; 512 pairs 0.52 / 0.73 / 1.19; 2048 pairs (one wave per SIMD
            // at R = 32) 1.44 at 32 against 1.50 at 8 and 1.82 at 16: chains of two R = 16 strips never
            // pay, so the choice is one strip per pair or R = 8 chains.
            const int64_t simds = 4 * (int64_t)std::max(1, num_cu);
            const int rc = knobs().pair_chain_r > 0 ? knobs().pair_chain_r : 8;
            const int64_t stripsC = (int64_t)((mmax + kWave * rc - 1) / (kWave * rc));
            if ((np / 2) * (int64_t)((mmax + kWave * r - 1) / (kWave * r)) < simds && r > rc && stripsC <= kPairChainMax)
                r = rc;
        }
        return r;
    }
    // few long pairs: the shortest strips keep the wavefront deepest (one row per lane)
    return 1;
}

// Waves per workgroup (strips per group). Chains of strips (pairs taller than one strip) hand
// their rows off through LDS inside a group; single-strip pairs gain nothing from grouping.
// band fill with persistent workers up to this many rows (DNA-sized alphabets / larger ones); past
// them the one-wave fill with one workgroup per CU is ahead (profiles/r05/ab_chain_per_cu_v0.log, ab_chain_solo_v1.log)
constexpr int64_t kBandPersistRows = 90112, kBandPersistRowsWide = 65536;

int choose_W(const std::vector<PairDesc> &pairs)
{
    const int w = knobs().waves_per_group;
    if (w >= 1 && w <= kMaxWaves) return w;
    (void)pairs;
    return 4;
}

void launch_fill(int R, const FillArgs &a, bool local, int sk, int grid, int W, bool chain, hipStream_t st)
{
    switch (R)
    {
    case 1: launch_fill_r<1>(a, local, sk, grid, W, chain, st); break;
    case 2: launch_fill_r<2>(a, local, sk, grid, W, chain, st); break;
    case 4: launch_fill_r<4>(a, local, sk, grid, W, chain, st); break;
    case 8: launch_fill_r<8>(a, local, sk, grid, W, chain, st); break;
    case 16: launch_fill_r<16>(a, local, sk, grid, W, chain, st); break;
    default: launch_fill_r<32>(a, local, sk, grid, W, chain, st); break;
    }
}

void free_plan(sa_plan *p)
{
    if (!p) return;
    if (p->borrowed) { delete p; return; }
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(p->device);
    void *bufs[] = {p->d_pairs, p->d_strips, p->d_prof, p->d_table, p->d_codes, p->d_masks, p->d_bnd,
                    p->d_best, p->d_score, p->d_ctrl, p->d_rec, p->d_heads, p->d_out_text,
                    p->d_out_pattern, p->d_results, p->d_bands, p->d_tbgroups, p->d_tbpg, p->d_tbl,
                    p->d_gtbl, p->d_gent, p->d_tbflag, p->d_csum, p->d_win, p->d_tbstart, p->d_sent,
                    p->d_sdelta, p->d_send, p->d_pend, p->d_cflag};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (p->own) (void)hipStreamDestroy(p->own);
    (void)hipSetDevice(cur);
    delete p;
}

int bitlen(uint64_t v)
{
    int b = 0;
    while (v) { ++b; v >>= 1; }
    return b;
}

// Compute units of `device`, cached (hipGetDeviceProperties costs milliseconds per call).
int device_cus(int device)
{
    static std::mutex mu;
    static std::vector<int> cus;
    std::lock_guard<std::mutex> lk(mu);
    if (device >= (int)cus.size()) cus.resize(device + 1, 0);
    if (cus[device] == 0)
    {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0)
        {
            (void)hipGetLastError();
            v = 256;
        }
        cus[device] = v;
    }
    return cus[device];
}

// Per-device state of the one-shot entry point (sa_align_pair, i.e. alignSequenceGPU): a stream,
// two timing events and a grow-only device arena that every call's plan and inputs are carved
// from, so a call costs its kernels and two small copies instead of ~16 hipMallocs, a stream
// creation and a device-property query (the reference re-allocates everything per call,
// alignSequenceGPU.cu:362-461). Calls on one device are serialised by `mu`; the arenas are
// released by sa_release_workspace or at process exit.
struct DeviceCtx {
    std::mutex mu;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    char *arena = nullptr;
    size_t arena_bytes = 0;
    // pinned host staging: a call's uploads leave in one DMA copy and its results come back in one
    // (pageable copies go through the runtime's staging blits, ~20 us each)
    char *pinned = nullptr;
    char *pinned_dev = nullptr;  // the same buffer as the kernels address it (stage_copy_kernel)
    size_t pinned_bytes = 0;
    // granules live in a buffer of their own (zeroed when allocated, never used for anything else)
    // and carry epochs that only grow across calls: a granule left by an earlier call never
    // matches, so the area needs no clearing per call. (Inside the shared arena it would: stale
    // records or scores there can look like a granule of the current epoch.)
    char *bnd = nullptr;
    size_t bnd_bytes = 0;
    uint32_t epoch = 0;
};

std::mutex g_ctx_mu;
std::vector<DeviceCtx *> g_ctx;

void release_ctx(DeviceCtx *c)
{
    std::lock_guard<std::mutex> lk(c->mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(c->device);
    if (c->arena) (void)hipFree(c->arena);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->bnd) (void)hipFree(c->bnd);
    c->bnd = nullptr;
    c->bnd_bytes = 0;
    c->pinned = nullptr;
    c->pinned_bytes = 0;
    if (c->e0) (void)hipEventDestroy(c->e0);
    if (c->e1) (void)hipEventDestroy(c->e1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    c->arena = nullptr;
    c->arena_bytes = 0;
    c->e0 = c->e1 = nullptr;
    c->stream = nullptr;
    (void)hipSetDevice(cur);
}

void release_all_ctx()
{
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    for (DeviceCtx *c : g_ctx)
        if (c) release_ctx(c);
}

// The context of `device` (created on first use; its stream and events too). Caller holds c->mu.
DeviceCtx *device_ctx(int device)
{
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if (device < 0 || device > 1024) return nullptr;
    if (device >= (int)g_ctx.size()) g_ctx.resize(device + 1, nullptr);
    if (!g_ctx[device])
    {
        if (g_ctx.size() == (size_t)device + 1 && std::all_of(g_ctx.begin(), g_ctx.end() - 1, [](DeviceCtx *c) { return !c; }))
            std::atexit(release_all_ctx);  // registered after HIP initialised: runs before its teardown
        g_ctx[device] = new DeviceCtx();
        g_ctx[device]->device = device;
    }
    return g_ctx[device];
}

// Makes sure c (locked by the caller, current device = c->device) has a stream, events and an
// arena of at least `bytes`.
int ctx_prepare(DeviceCtx *c, size_t bytes)
{
    if (!c->stream) HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!c->e0) HIP_TRY(hipEventCreate(&c->e0));
    if (!c->e1) HIP_TRY(hipEventCreate(&c->e1));
    if (c->arena_bytes < bytes)
    {
        // grow geometrically (x1.25 of the old size) so a sweep of rising sizes does not reallocate
        // every call
        const size_t want = std::max(bytes, c->arena_bytes + c->arena_bytes / 4);
        if (c->arena)
        {
            HIP_TRY(hipStreamSynchronize(c->stream));
            (void)hipFree(c->arena);
            c->arena = nullptr;
            c->arena_bytes = 0;
        }
        if (hipMalloc((void **)&c->arena, want) != hipSuccess)
        {
            (void)hipGetLastError();
            c->arena = nullptr;
            if (want == bytes || hipMalloc((void **)&c->arena, bytes) != hipSuccess)
            {
                (void)hipGetLastError();
                c->arena = nullptr;
                return fail(SA_ERR_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes failed");
            }
            c->arena_bytes = bytes;
        }
        else c->arena_bytes = want;
    }
    return SA_OK;
}

// Makes sure c has a granule buffer of at least `bytes` (zeroed when (re)allocated).
int ctx_bnd(DeviceCtx *c, size_t bytes)
{
    if (c->bnd_bytes >= bytes) return SA_OK;
    if (c->bnd)
    {
        HIP_TRY(hipStreamSynchronize(c->stream));
        (void)hipFree(c->bnd);
        c->bnd = nullptr;
        c->bnd_bytes = 0;
    }
    const size_t want = std::max(bytes, (size_t)1 << 16);
    if (hipMalloc((void **)&c->bnd, want) != hipSuccess)
    {
        (void)hipGetLastError();
        c->bnd = nullptr;
        return fail(SA_ERR_NOMEM, "device allocation of " + std::to_string(want) + " bytes failed");
    }
    c->bnd_bytes = want;
    HIP_TRY(hipMemsetAsync(c->bnd, 0, want, c->stream));
    return SA_OK;
}

// Makes sure c has a pinned staging buffer of at least `bytes`.
int ctx_pinned(DeviceCtx *c, size_t bytes)
{
    if (c->pinned_bytes >= bytes) return SA_OK;
    if (c->pinned)
    {
        HIP_TRY(hipStreamSynchronize(c->stream));
        (void)hipHostFree(c->pinned);
        c->pinned = nullptr;
        c->pinned_bytes = 0;
    }
    const size_t want = std::max(bytes, (size_t)1 << 20);
    HIP_TRY(hipHostMalloc((void **)&c->pinned, want, hipHostMallocDefault));
    HIP_TRY(hipHostGetDevicePointer((void **)&c->pinned_dev, c->pinned, 0));
    c->pinned_bytes = want;
    return SA_OK;
}

// One-shot calls move their staging blob through the pinned buffer with a kernel on the call's
// stream instead of a DMA copy: the copy engine's hand-off to and from the compute queue cost ≈ 10 us
// each way per call (rocprofv3 memory-copy trace of the latency mode, profiles/r06/latency_*), the
// kernel reads or writes the host buffer directly over the fabric. 16-byte vector loads and stores;
// the last bytes one at a time. (SA_STAGE_KERNEL=0: the DMA copies.)
__global__ __launch_bounds__(256) void stage_copy_kernel(char *dst, const char *src, uint64_t bytes)
{
    const uint64_t n16 = bytes / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
    if (blockIdx.x == 0 && threadIdx.x < bytes % 16) dst[16 * n16 + threadIdx.x] = src[16 * n16 + threadIdx.x];
}

hipError_t stage_copy(char *dst, const char *src, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    const uint64_t n16 = bytes / 16 + 1;
    const int grid = (int)std::min<uint64_t>(1024, (n16 + 255) / 256);
    hipLaunchKernelGGL(stage_copy_kernel, dim3(grid), dim3(256), 0, st, dst, src, (uint64_t)bytes);
    return hipGetLastError();
}

constexpr size_t kArenaAlign = 256;
size_t arena_round(size_t b) { return (std::max<size_t>(b, 16) + kArenaAlign - 1) / kArenaAlign * kArenaAlign; }

// host inputs a workspace plan uploads together with its descriptors (sa_align_pair)
struct OneShotInputs {
    const char *text = nullptr, *pattern = nullptr;
    uint64_t n = 0, m = 0;
};
int plan_create(const sa_params *P, const sa_pair *pairs, int64_t np, int device, DeviceCtx *ws,
                const OneShotInputs *in, sa_plan **out);

}  // namespace

extern "C" {

const char *sa_last_error(void) { return g_err.c_str(); }
int sa_abi_version(void) { return SA_ABI_VERSION; }

int sa_device_count(int *count)
{
    HIP_TRY(hipGetDeviceCount(count));
    return SA_OK;
}

int sa_plan_create(const sa_params *P, const sa_pair *pairs, int64_t np, int device, sa_plan **out)
{
    return plan_create(P, pairs, np, device, nullptr, nullptr, out);
}

}  // extern "C"

namespace {

// Builds a plan. With `ws` (a locked DeviceCtx, current device set) every device buffer is carved
// from the context's arena, the host inputs `in` too, and everything the fill reads from the host
// goes up in one asynchronous copy from the context's pinned buffer; otherwise buffers are
// hipMalloc'd and uploaded one by one.
int plan_create(const sa_params *P, const sa_pair *pairs, int64_t np, int device, DeviceCtx *ws,
                const OneShotInputs *in, sa_plan **out)
{
    if (!P || !out || np < 0 || (np > 0 && !pairs) || !P->score_matrix)
        return fail(SA_ERR_INVALID, "sa_plan_create: null argument");
    *out = nullptr;
    const int A = P->alphabet_size;
    if (A < 1 || A > 32) return fail(SA_ERR_INVALID, "alphabet_size must be 1..32");
    if (P->mode != SA_GLOBAL && P->mode != SA_LOCAL) return fail(SA_ERR_INVALID, "mode must be SA_GLOBAL or SA_LOCAL");
    // any int gap penalty, as the reference's CLI (std::stoi, utilities.cpp:188-199) and its fill
    // (alignSequenceCPU.cpp:175-176, 259-260) take it; the range bound below rejects what int32 cannot hold
    const int64_t g = P->gap_penalty;
    int64_t smax = INT32_MIN, smin = INT32_MAX, sabs = 0;
    for (int e = 0; e < A * A; ++e)
    {
        smax = std::max<int64_t>(smax, P->score_matrix[e]);
        smin = std::min<int64_t>(smin, P->score_matrix[e]);
        sabs = std::max<int64_t>(sabs, std::llabs((long long)P->score_matrix[e]));
    }
    // numeric limits of the engine: every intermediate fits in int32, local keys fit.
    uint64_t hmax_local = 0, lmax = 0;
    for (int64_t p = 0; p < np; ++p)
    {
        const uint64_t n = pairs[p].text_len, m = pairs[p].pattern_len;
        if (n >= (1u << 24) - 1 || m >= (1u << 24) - 1)
            return fail(SA_ERR_UNSUPPORTED, "sequence longer than 2^24-2 letters");
        lmax = std::max(lmax, std::max(n, m));
        const uint64_t span = n + m;
        const uint64_t bound = ((uint64_t)sabs + (uint64_t)std::llabs(g)) * span + (uint64_t)std::llabs(g) * span;
        if (bound >= (1ull << 30)) return fail(SA_ERR_UNSUPPORTED, "scores may exceed the int32 range");
        const uint64_t h = g >= 0 ? (uint64_t)std::max<int64_t>(smax, 0) * std::min(n, m)
                                  : ((uint64_t)sabs + (uint64_t)(-g)) * span;
        hmax_local = std::max(hmax_local, h);
    }
    // local best-cell keys: H | ~row | ~col in 64 bits, row / column fields sized for the longest
    // sequence; the in-kernel block key (H << key_bits) + step must stay inside int32
    const int key_rowbits = std::max(1, bitlen(lmax + 1));
    if (P->mode == SA_LOCAL && (bitlen(hmax_local) > 26 || bitlen(hmax_local) > 64 - 2 * key_rowbits))
        return fail(SA_ERR_UNSUPPORTED, "local scores may exceed the best-cell key range");

    sa_plan *pl = new sa_plan();
    pl->device = device;
    pl->mode = P->mode;
    pl->A = A;
    pl->gap = (int)g;
    pl->R = choose_R(P, pairs, np, knobs().max_cus > 0 ? std::min(device_cus(device), knobs().max_cus) : device_cus(device));
    pl->U = (16 / pl->R) > 4 ? 16 / pl->R : 4;
    pl->key_bits = std::min(12, std::max(4, 30 - bitlen(hmax_local)));
    pl->key_rowbits = key_rowbits;
    // the tables hold S + 2g (global, shifted domain) or S + g (local), see run_body
    const int64_t off2 = P->mode == SA_GLOBAL ? 2 * g : g;
    bool fits8 = true;
    for (int e = 0; e < A * A; ++e)
    {
        const int64_t v = P->score_matrix[e] + off2;
        if (v < -128 || v > 127) fits8 = false;
    }
    // kArr8's hand-scheduled bodies keep the direction differences in bytes (sa_fill_steps.inc): every
    // |M - D|, |left - up| is at most 2 (|S| + 2|g|) (global, shifted domain: every boundary is 0 and
    // adjacent cells differ by at most max(S + 2g, 0)) or 2 (|S| + |g|) + |g| (local, g >= 0), below
    // 4 (max|S| + |g|). Local with g < 0 has no such bound: H(i, 1) grows like -g * i next to the
    // column-0 zeros, so M - D at column 1 (and row 1) leaves the byte range.
    const bool byte_diffs = 4 * (sabs + std::llabs(g)) <= 127 && !(P->mode == SA_LOCAL && g < 0);
    if (pl->R == 1) pl->sk = fits8 && byte_diffs ? kArr8 : kArr;
    else pl->sk = (A <= 4 && fits8) ? kProf : kTable;
    if (P->alphabet) std::memcpy(pl->alphabet, P->alphabet, std::min<size_t>(A + 1, 33));
    else for (int c = 0; c <= A; ++c) pl->alphabet[c] = c == A ? '-' : (char)('A' + c);

    int cur = 0;
    (void)hipGetDevice(&cur);
    auto restore = [&]() { (void)hipSetDevice(cur); };
    if (hipSetDevice(device) != hipSuccess) { delete pl; restore(); return fail(SA_ERR_HIP, "hipSetDevice failed"); }
    pl->num_cu = device_cus(device);
    if (knobs().max_cus > 0) pl->num_cu = std::min(pl->num_cu, knobs().max_cus);

    // ---- layout ----
    const int R = pl->R, U = pl->U, RB = kWave * R;
    uint64_t code_bytes = 0, mask_entries = 0, granules = 0, outb = 0, recw = 0;
    pl->pairs.resize(np);
    for (int64_t p = 0; p < np; ++p)
    {
        PairDesc &d = pl->pairs[p];
        d.text_off = pairs[p].text_offset;
        d.text_len = pairs[p].text_len;
        d.pattern_off = pairs[p].pattern_offset;
        d.pattern_len = pairs[p].pattern_len;
        d.code_off = code_bytes;
        // kArr8: code_len bytes per copy (4A copies); kArr: A arrays of code_len dwords; else one
        d.code_len = (kPad + d.text_len + 4 * kPad + 3) / 4 * 4;
        // (a possible pair-packed plan, decided below, needs two column profiles per column)
        const bool maybePair = P->mode == SA_GLOBAL && R >= 4 && A <= 4;
        code_bytes += pl->sk == kArr8 ? (uint64_t)A * d.code_len : pl->sk == kArr ? (uint64_t)A * d.code_len
                                                                                : (maybePair ? 2 : 1) * d.code_len;
        d.out_off = outb;
        outb += d.text_len + d.pattern_len + 16;
        d.rec_off = recw;
        recw += std::max(d.text_len, d.pattern_len) + 64;
        d.first_strip = (int32_t)pl->strips.size();
        const uint64_t n = d.text_len, m = d.pattern_len;
        const int ns = (n == 0 || m == 0) ? 0 : (int)((m + RB - 1) / RB);
        d.num_strips = ns;
        // n + 63 steps reach column n in lane 63; one more step moves its bottom-row value into the
        // publishing register (sa_fill.hip run_body); two bodies per loop trip
        const int nsteps = (int)(((n + kWave) + 2 * U - 1) / (2 * U) * (2 * U));
        for (int b = 0; b < ns; ++b)
        {
            StripDesc s;
            s.pair = (int32_t)p;
            s.row0 = 1 + b * RB;
            s.flags = (b > 0 ? kHasPrev : 0) | (b + 1 < ns ? kHasNext : 0);
            s.nsteps = nsteps;
            s.mask_off = mask_entries;
            mask_entries += (uint64_t)nsteps * R;
            s.bnd_in = b > 0 ? pl->strips.back().bnd_out : 0;
            s.bnd_out = granules;
            if (b + 1 < ns) granules += n + 8;
            pl->strips.push_back(s);
        }
    }
    if (pl->strips.size() >= (1u << 31)) { delete pl; restore(); return fail(SA_ERR_UNSUPPORTED, "too many strips"); }
    pl->out_bytes = outb;
    pl->bytes_masks = mask_entries * 16;
    pl->W = choose_W(pl->pairs);
    for (const PairDesc &d : pl->pairs) pl->chain = pl->chain || d.num_strips > 1;
    {
        // pair-packed fill: global, pairs of one shape, DNA-sized alphabet, every S + 2g in [0, 255]
        // and every value within u16 (see process_pair). Lone strips: fill_pair_kernel; chains of up
        // to kPairChainMax strips per pair (every pair the same count): fill_pair_chain_kernel, one
        // workgroup per couple, its LDS rows within a CU's
        bool pair = R >= 4 && pair_packable(P, pairs, np);
        if (pair && pl->chain)
        {
            const int S = pl->pairs[0].num_strips;
            pair = S <= kPairChainMax && (size_t)(S - 1) * pair_row_entries((int)pl->pairs[0].text_len) * 4 <= 160 * 1024;
        }
        if (pair)
        {
            pl->sk = kPair;
            granules = 0;  // (the chains hand their rows off in LDS: no granules)
        }
    }
    // the band fill (sa_fill.hip process_band): R = 1 chains with int8 text profiles (global, or local
    // with g >= 0, which kArr8 implies), W even (a group boundary inside a pair must fall on a band
    // boundary: every pair's first strip even), and the band groups plus the strip groups fit one
    // workgroup per CU
    {
        bool band = knobs().band != 0 && pl->R == 1 && pl->sk == kArr8 && pl->chain && pl->W % 2 == 0;
        for (const PairDesc &d : pl->pairs) band = band && (d.num_strips == 0 || d.first_strip % 2 == 0);
        int64_t nb = 0;
        for (const PairDesc &d : pl->pairs) nb += std::max(0, (d.num_strips + 1) / 2 - 1);
        const int64_t stripGroups = ((int64_t)pl->strips.size() + pl->W - 1) / pl->W;
        const int64_t bandGroups = (nb + pl->W - 1) / pl->W;
        // every group in flight at once, or (persistent band and strip workgroups, FillArgs::band_wgs)
        // chains up to kBandPersistRows rows: past them the fill is throughput-bound and the bands' work
        // on top of the strips' costs more than their shorter ramp saves
        int64_t mmax = 0;
        for (const PairDesc &d : pl->pairs) mmax = std::max<int64_t>(mmax, (int64_t)d.pattern_len);
        const int64_t persistRows = knobs().band_rows > 0 ? knobs().band_rows : (A <= 4 ? kBandPersistRows : kBandPersistRowsWide);
        band = band && nb > 0 &&
               (stripGroups + bandGroups <= pl->num_cu || ((mmax <= persistRows || knobs().band == 1) && pl->num_cu >= 4));
        if (band)
        {
            // bands b = 0 .. B-2 of each pair (B = ceil(strips / 2); the last band's bottom row feeds
            // nothing); every band publishes its bottom row to granules. The strips keep their planes;
            // a strip at a group start takes its feed from the granules of the band above, the others
            // from the strip above through the group's rings, and a group's last strip publishes nothing.
            granules = 0;
            for (const PairDesc &d : pl->pairs)
            {
                const uint64_t n = d.text_len;
                const int B = (d.num_strips + 1) / 2;
                const int64_t fb = (int64_t)pl->bands.size();
                for (int b = 0; b + 1 < B; ++b)
                {
                    StripDesc bd = pl->strips[d.first_strip + 2 * b];
                    bd.row0 = 1 + b * 2 * kWave;
                    bd.flags = (b > 0 ? kHasPrev : 0) | kHasNext;
                    bd.mask_off = 0;
                    bd.bnd_in = b > 0 ? pl->bands.back().bnd_out : 0;
                    bd.bnd_out = granules;
                    granules += n + 8;
                    pl->bands.push_back(bd);
                }
                for (int k = 0; k < d.num_strips; ++k)
                {
                    StripDesc &sd = pl->strips[d.first_strip + k];
                    const int i = d.first_strip + k;
                    if (k + 1 < d.num_strips && (i + 1) % pl->W == 0) sd.flags &= ~kHasNext;
                    sd.bnd_out = 0;
                    sd.bnd_in = (k > 0 && i % pl->W == 0) ? pl->bands[fb + k / 2 - 1].bnd_out : 0;
                }
            }
            pl->band = true;
        }
    }
    {
        // one-wave chain fill: a second workgroup on a CU puts two compute waves on a SIMD, which
        // raises the step time 25 -> 41 ns and the hand-off lag 2.5 -> 4.6 us (tools/timeline.py,
        // 120000^2); the strip chains of a few long pairs are latency-bound (a strip starts one lag
        // after the one above), so they get one workgroup per CU; many chained pairs keep two
        int64_t chained = 0;
        for (const PairDesc &d : pl->pairs) chained += d.num_strips > 1;
        pl->chain_solo = pl->chain && !pl->band && chained < pl->num_cu;
        if (knobs().chain_per_cu) pl->chain_solo = pl->chain && !pl->band && knobs().chain_per_cu == 1;
    }

    // ---- tables ----
    std::vector<int32_t> &prof = pl->h_prof, &table = pl->h_table;
    prof.assign(4, 0);
    table.resize(A * A);
    for (int e = 0; e < A * A; ++e) table[e] = (int32_t)(P->score_matrix[e] + off2);
    if (pl->sk == kProf || pl->sk == kPair)
        for (int cp = 0; cp < A; ++cp)
        {
            uint32_t w = 0;
            for (int ct = 0; ct < A; ++ct) w |= (uint32_t)(table[cp * A + ct] & 0xff) << (8 * ct);
            prof[cp] = (int32_t)w;
        }

    // ---- table traceback groups (sa_walk.h) ----
    if (pl->R == 1 && knobs().tb_tables)
    {
        pl->tb_pg.assign(np + 1, 0);
        for (int64_t p = 0; p < np; ++p)
        {
            const PairDesc &d = pl->pairs[p];
            pl->tb_pg[p] = (int32_t)pl->tb_groups.size();
            if (d.num_strips < kTbMinStrips || d.text_len == 0) continue;
            // strip tables only for the strips of pairs with groups (slot tbl0 + s - s_lo)
            for (int s = 0; s < d.num_strips; s += kTbG)
                pl->tb_groups.push_back({(int32_t)p, d.first_strip + s, d.first_strip + std::min(d.num_strips, s + kTbG) - 1,
                                         (int32_t)pl->tb_slots + s});
            pl->tb_slots += d.num_strips;
        }
        pl->tb_pg[np] = (int32_t)pl->tb_groups.size();
        if (pl->tb_groups.empty()) pl->tb_pg.clear();
    }
    const size_t ntg = pl->tb_groups.size();
    for (const PairDesc &d : pl->pairs)
        pl->max_recs = std::max<int64_t>(pl->max_recs, (int64_t)(pl->R == 1 ? d.pattern_len : d.text_len));

    // ---- device buffers ----
    const size_t nstr = std::max<size_t>(1, pl->strips.size()), npp = std::max<size_t>(1, np);
    const size_t codeB = 4 * code_bytes + 16, bndB = granules * 8 + 16, bestB = sizeof(uint64_t) * nstr;
    struct Buf { void **ptr; size_t bytes; };
    const uint64_t inN = in ? in->n : 0, inM = in ? in->m : 0;
    // order matters for workspace plans: [pairs .. ctrl] is the upload region, [ctrl .. out_pattern]
    // the download region (zero-sized entries are skipped)
    const Buf bufs[] = {
        {(void **)&pl->d_pairs, sizeof(PairDesc) * npp},
        {(void **)&pl->d_strips, sizeof(StripDesc) * nstr},
        {(void **)&pl->d_prof, sizeof(int32_t) * 4},
        {(void **)&pl->d_table, sizeof(int32_t) * A * A},
        {(void **)&pl->d_bands, sizeof(StripDesc) * pl->bands.size()},
        {(void **)&pl->d_tbgroups, sizeof(TbGroup) * ntg},
        {(void **)&pl->d_tbpg, ntg ? sizeof(int32_t) * (np + 1) : 0},
        {(void **)&pl->d_ws_text, in ? inN + 16 : 0},
        {(void **)&pl->d_ws_pattern, in ? inM + 16 : 0},
        {(void **)&pl->d_ctrl, sizeof(Control)},
        {(void **)&pl->d_results, sizeof(sa_result) * npp},
        {(void **)&pl->d_out_text, outb + 16},
        {(void **)&pl->d_out_pattern, outb + 16},
        {(void **)&pl->d_codes, codeB},
        // (+8 KiB: the traceback's plane prefetch may read a few chunks past a strip)
        {(void **)&pl->d_masks, pl->bytes_masks + 8192},
        {(void **)&pl->d_bnd, ws ? 0 : bndB},  // (workspace plans: the context's granule buffer)
        {(void **)&pl->d_best, bestB},
        {(void **)&pl->d_score, sizeof(int32_t) * npp},
        {(void **)&pl->d_rec, 4 * recw + 16},
        {(void **)&pl->d_heads, sizeof(TbHead) * npp},
        {(void **)&pl->d_tbl, ntg ? sizeof(int32_t) * kTbK * pl->tb_slots : 0},
        {(void **)&pl->d_gtbl, sizeof(int32_t) * kTbK * ntg},
        {(void **)&pl->d_gent, sizeof(int32_t) * ntg},
        {(void **)&pl->d_tbflag, ntg ? sizeof(int32_t) * npp : 0},
        {(void **)&pl->d_win, ntg ? sizeof(int32_t) * nstr : 0},
        {(void **)&pl->d_tbstart, ntg ? sizeof(int32_t) * kTbStartWords * npp : 0},
        {(void **)&pl->d_pend, ntg ? sizeof(int32_t) * npp : 0},
        {(void **)&pl->d_sent, ntg && P->mode == SA_LOCAL ? sizeof(int32_t) * nstr : 0},
        {(void **)&pl->d_sdelta, ntg && P->mode == SA_LOCAL ? sizeof(int32_t) * nstr : 0},
        {(void **)&pl->d_send, ntg && P->mode == SA_LOCAL ? sizeof(int32_t) * 4 * nstr : 0},
        {(void **)&pl->d_csum, pl->max_recs > kChunkRecs ? sizeof(int64_t) * kMaxChunks * npp : 0},
        {(void **)&pl->d_cflag, pl->max_recs > kChunkRecs ? sizeof(uint64_t) * kMaxChunks * npp : 0},
    };
    int rc = SA_OK;
    if (ws)
    {
        size_t total = 0;
        for (const Buf &b : bufs) total += b.bytes ? arena_round(b.bytes) : 0;
        if ((rc = ctx_prepare(ws, total)) != SA_OK) { delete pl; restore(); return rc; }
        size_t off = 0;
        for (const Buf &b : bufs)
        {
            if (!b.bytes) continue;
            *b.ptr = ws->arena + off;
            off += arena_round(b.bytes);
        }
        if ((rc = ctx_bnd(ws, bndB)) != SA_OK) { delete pl; restore(); return rc; }
        pl->d_bnd = (uint64_t *)ws->bnd;
        pl->bytes_total = total + bndB;
        pl->borrowed = true;
        pl->own = ws->stream;
        pl->epoch_src = &ws->epoch;
        pl->d_up = (char *)pl->d_pairs;
        pl->up_bytes = (size_t)((char *)pl->d_ctrl - pl->d_up) + sizeof(Control);
        pl->d_dn = (char *)pl->d_ctrl;
        pl->dn_bytes = (size_t)(pl->d_out_pattern - pl->d_dn) + outb + 16;
        if ((rc = ctx_pinned(ws, std::max(pl->up_bytes, pl->dn_bytes))) != SA_OK) { delete pl; restore(); return rc; }
        // one upload: descriptors, tables, the inputs and a zeroed control word at their arena
        // offsets. The code block is written whole by the encode kernel, granules carry growing
        // epochs in their own buffer (DeviceCtx) and every strip writes its best key, so nothing
        // else needs clearing.
        char *h = ws->pinned;
        auto put = [&](const void *dptr, const void *src, size_t bytes) {
            if (bytes) std::memcpy(h + ((const char *)dptr - pl->d_up), src, bytes);
        };
        put(pl->d_pairs, pl->pairs.data(), sizeof(PairDesc) * np);
        put(pl->d_strips, pl->strips.data(), sizeof(StripDesc) * pl->strips.size());
        put(pl->d_prof, prof.data(), sizeof(int32_t) * 4);
        put(pl->d_table, table.data(), sizeof(int32_t) * A * A);
        put(pl->d_bands, pl->bands.data(), sizeof(StripDesc) * pl->bands.size());
        put(pl->d_tbgroups, pl->tb_groups.data(), sizeof(TbGroup) * ntg);
        if (ntg) put(pl->d_tbpg, pl->tb_pg.data(), sizeof(int32_t) * (np + 1));
        put(pl->d_ws_text, in->text, inN);
        put(pl->d_ws_pattern, in->pattern, inM);
        std::memset(h + ((char *)pl->d_ctrl - pl->d_up), 0, sizeof(Control));
        if ((knobs().stage_kernel ? stage_copy(pl->d_up, ws->pinned_dev, pl->up_bytes, pl->own)
                                  : hipMemcpyAsync(pl->d_up, h, pl->up_bytes, hipMemcpyHostToDevice, pl->own)) != hipSuccess)
        {
            free_plan(pl);
            restore();
            return fail(SA_ERR_HIP, "plan upload failed");
        }
        pl->ctrl_ready = true;
        restore();
        *out = pl;
        return SA_OK;
    }
    for (const Buf &b : bufs)
        if (rc == SA_OK && b.bytes) { rc = dmalloc(b.ptr, b.bytes); pl->bytes_total += b.bytes; }
    if (rc != SA_OK) { free_plan(pl); restore(); return rc; }
    if (hipStreamCreateWithFlags(&pl->own, hipStreamNonBlocking) != hipSuccess) { free_plan(pl); restore(); return fail(SA_ERR_HIP, "stream creation failed"); }
    // uploads (asynchronous on the plan's stream; the host sources live in the plan)
    hipStream_t st = pl->own;
    bool okc = hipMemcpyAsync(pl->d_pairs, pl->pairs.data(), sizeof(PairDesc) * np, hipMemcpyHostToDevice, st) == hipSuccess &&
               hipMemcpyAsync(pl->d_strips, pl->strips.data(), sizeof(StripDesc) * pl->strips.size(), hipMemcpyHostToDevice, st) == hipSuccess &&
               hipMemcpyAsync(pl->d_prof, prof.data(), sizeof(int32_t) * 4, hipMemcpyHostToDevice, st) == hipSuccess &&
               hipMemcpyAsync(pl->d_table, table.data(), sizeof(int32_t) * A * A, hipMemcpyHostToDevice, st) == hipSuccess &&
               hipMemsetAsync(pl->d_bnd, 0, bndB, st) == hipSuccess &&
               hipMemsetAsync(pl->d_best, 0, bestB, st) == hipSuccess &&
               hipMemsetAsync(pl->d_ctrl, 0, sizeof(Control), st) == hipSuccess;  // (bad_input: no stale epoch)
    // expansion flags carry the plan's epoch, which starts again at 1 for a plan of its own: a freed
    // plan's flags at the same address would match (workspace plans draw epochs from their device's
    // context, which only grow, so their arena needs no clearing)
    if (okc && pl->d_cflag)
        okc = hipMemsetAsync(pl->d_cflag, 0, sizeof(uint64_t) * kMaxChunks * npp, st) == hipSuccess;
    if (okc && pl->band)
        okc = hipMemcpyAsync(pl->d_bands, pl->bands.data(), sizeof(StripDesc) * pl->bands.size(), hipMemcpyHostToDevice, st) == hipSuccess;
    if (okc && ntg)
        okc = hipMemcpyAsync(pl->d_tbgroups, pl->tb_groups.data(), sizeof(TbGroup) * ntg, hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemcpyAsync(pl->d_tbpg, pl->tb_pg.data(), sizeof(int32_t) * (np + 1), hipMemcpyHostToDevice, st) == hipSuccess;
    // a plan of its own is complete when sa_plan_create returns (callers fill on other streams)
    if (okc) okc = hipStreamSynchronize(st) == hipSuccess;
    if (!okc) { free_plan(pl); restore(); return fail(SA_ERR_HIP, "plan upload failed"); }
    restore();
    *out = pl;
    return SA_OK;
}

}  // namespace

extern "C" {

int sa_plan_destroy(sa_plan *plan)
{
    free_plan(plan);
    return SA_OK;
}

int sa_plan_fill(sa_plan *pl, const void *d_text, const void *d_pattern, void *stream)
{
    if (!pl || (!pl->pairs.empty() && (!d_text || !d_pattern))) return fail(SA_ERR_INVALID, "sa_plan_fill: null argument");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    pl->d_text_in = (const int8_t *)d_text;
    pl->d_pattern_in = (const int8_t *)d_pattern;
    uint32_t *es = pl->epoch_src ? pl->epoch_src : &pl->epoch;
    if (++*es == 0) ++*es;
    pl->epoch = *es;
    // A plan of one pair leaves the reset of its control word to the encode kernel below; plans of
    // several pairs keep the memset launch: without it the pipelined batch step (two plans, the fill
    // and the traceback on two streams) went from 2.45 to 3.34 ms, while the same reset with the
    // launch kept measured 2.45 (profiles/r06/ab_ctrl_reset_diagnosis_v1.log)
    if (!pl->ctrl_ready && pl->pairs.size() != 1) HIP_TRY(hipMemsetAsync(pl->d_ctrl, 0, sizeof(Control), st));
    pl->ctrl_ready = false;
    const int np = (int)pl->pairs.size();
    if (np > 0)
    {
        uint64_t nmax = 1;
        for (auto &d : pl->pairs) nmax = std::max<uint64_t>(nmax, std::max(d.text_len, d.pattern_len));
        // (text profiles: one thread per dword and alphabet row)
        const uint64_t work = pl->sk == kArr8 ? (nmax / 4 + kPad) * (uint64_t)pl->A : nmax;
        // at most ~8192 blocks in all: many small pairs loop inside their blocks rather than paying
        // for block dispatch (4096 pairs x 8 blocks took 50 us, mostly dispatch)
        const int gx = (int)std::min<uint64_t>((work + 255) / 256, std::max(1, std::min(1024, 8192 / np)));
        for (int y0 = 0; y0 < np; y0 += 65534)
        {
            // pairs beyond 65535 are handled by re-basing the pair pointer
            const int cnt = std::min(65534, np - y0);  // even: kPair pairs (2q, 2q+1) stay in one launch
            hipLaunchKernelGGL(encode_text_kernel, dim3(gx, cnt), dim3(256), 0, st, (const int8_t *)d_text,
                               (const int8_t *)d_pattern, pl->d_pairs + y0, pl->d_codes, pl->A, pl->sk, pl->d_table,
                               pl->d_ctrl, pl->epoch);
        }
        HIP_TRY(hipGetLastError());
        if (int rc = debug_sync(st, "encode_text_kernel")) return rc;
    }
    const int ns = (int)pl->strips.size();
    if (ns > 0)
    {
        FillArgs a;
        a.pattern = (const int8_t *)d_pattern;
        a.codes = pl->d_codes;
        a.strips = pl->d_strips;
        a.pairs = pl->d_pairs;
        a.prof_tab = pl->d_prof;
        a.score_tab = pl->d_table;
        a.masks = pl->d_masks;
        a.bnd = pl->d_bnd;
        a.strip_best = pl->d_best;
        a.pair_score = pl->d_score;
        a.ctrl = pl->d_ctrl;
        a.num_strips = ns;
        a.gap = pl->gap;
        a.A = pl->A;
        a.epoch = pl->epoch;
        a.key_bits = pl->key_bits;
        a.key_rowbits = pl->key_rowbits;
        a.timeout_ticks = (uint64_t)(knobs().handoff_timeout_s * 1e8);
        a.io_sleep = knobs().io_sleep;
        a.chain_lds = knobs().chain_lds_kb * 1024;
        a.bands = pl->d_bands;
        a.num_bands = 0;
        a.num_band_groups = 0;
        a.band_wgs = 0;
        a.pair_text_len = 0;
        // SA_TIMELINE=<file>: debug dump of per-strip timestamps (s_memrealtime, 100 MHz)
        const char *tlPath = knobs().timeline;
        a.timeline = nullptr;
        DevPtr<uint64_t> tlBuf;
        if (tlPath)
        {
            HIP_TRY(hipMalloc((void **)&a.timeline, sizeof(uint64_t) * kTimelineWords * (ns + pl->bands.size())));
            tlBuf.reset(a.timeline);
        }
        // (the pair-packed kernel always runs kPairWaves waves per workgroup)
        const int W = pl->sk == kPair ? kPairWaves : pl->W;
        a.num_groups = (ns + W - 1) / W;
        // chains: two workgroups of W compute waves + an I/O wave per CU; lone strips: W compute
        // waves per workgroup and up to 16 waves per CU (the batch kernel stays under 128 VGPRs)
        const int perCU = pl->chain ? std::max(1, 8 / W) : std::max(1, 16 / W);
        int grid = std::min(a.num_groups, std::max(1, pl->num_cu) * perCU);
        if (pl->sk == kPair)
        {
            // one wave per two strips
            const int units = ns / 2;
            a.num_groups = (units + W - 1) / W;
            grid = std::min(a.num_groups, std::max(1, pl->num_cu) * std::max(1, 8 / W));
        }
        if (pl->sk == kPair && pl->chain)
        {
            // pair-packed chains: one workgroup per couple of pairs, one wave per strip of the couple
            a.num_groups = ns / 2 / pl->pairs[0].num_strips;
            a.pair_text_len = (int32_t)pl->pairs[0].text_len;
            grid = a.num_groups;
        }
        else if (pl->chain_solo)
        {
            // (plan_create) an LDS request above half a CU's keeps a second workgroup off the CU
            a.chain_lds = std::max(a.chain_lds, 96 * 1024);
            grid = std::min(a.num_groups, std::max(1, pl->num_cu));
        }
        if (pl->band)
        {
            // band groups on the first workgroups, strip groups on the rest, one workgroup per CU (the
            // LDS request is above half a CU's) and every group in flight at once (plan_create checked
            // that they fit): a strip group waits only for bands, which never wait for strips
            a.num_bands = (int32_t)pl->bands.size();
            a.num_band_groups = (a.num_bands + W - 1) / W;
            a.band_wgs = a.num_band_groups;
            a.chain_lds = std::max(a.chain_lds, 96 * 1024);
            grid = a.num_band_groups + a.num_groups;
            if (grid > pl->num_cu)
            {
                // more groups than CUs: persistent workers, each taking groups from its queue in chain
                // order until it is empty (a group waits only for groups dequeued before it, so every
                // worker count makes progress); the split that a model of the band and strip chains
                //  puts ahead for 65536^2 .. 120000^2 is about 0.31 of the CUs to bands
                a.band_wgs = std::max(1, std::min(a.num_band_groups, (int)(0.31 * pl->num_cu + 0.5)));
                grid = a.band_wgs + std::max(1, std::min(a.num_groups, pl->num_cu - a.band_wgs));
            }
        }
        // chains of protein-sized alphabets read copy 0 of their text profiles (kArr8A, sa_fill.h)
        const int sk = pl->sk == kArr8 && pl->chain && knobs().align > (pl->A > 4 ? 0 : 1) ? kArr8A : pl->sk;
        launch_fill(pl->R, a, pl->mode == SA_LOCAL, sk, grid, pl->sk == kPair && pl->chain ? pl->pairs[0].num_strips : W,
                    pl->chain, st);
        HIP_TRY(hipGetLastError());
        if (tlPath)
        {
            std::vector<uint64_t> tl(kTimelineWords * (ns + pl->bands.size()));
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipMemcpy(tl.data(), a.timeline, tl.size() * 8, hipMemcpyDeviceToHost));
            if (FILE *f = std::fopen(tlPath, "wb"))
            {
                std::fwrite(tl.data(), 8, tl.size(), f);
                std::fclose(f);
            }
        }
        if (int rc = debug_sync(st, "fill_kernel")) return rc;
    }
    pl->filled = true;
    return SA_OK;
}

int sa_plan_traceback(sa_plan *pl, void *stream)
{
    if (!pl || !pl->filled) return fail(SA_ERR_INVALID, "sa_plan_traceback: plan not filled");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    const int np = (int)pl->pairs.size();
    if (np == 0) return SA_OK;
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    const Knobs &kn = knobs();
    // SA_TB_TIMING=<file>: debug dump of per-pair phase timestamps (s_memrealtime, 100 MHz)
    const char *tmPath = kn.tb_timing;
    uint64_t *timing = nullptr;
    DevPtr<uint64_t> tmBuf;
    if (tmPath)
    {
        HIP_TRY(hipMalloc((void **)&timing, sizeof(uint64_t) * 9 * np));
        tmBuf.reset(timing);
    }
    // row / column walk (records) + expansion (sa_walk.hip)
    WalkArgs w;
    w.strips = pl->d_strips;
    w.pairs = pl->d_pairs;
    w.masks = pl->d_masks;
    w.strip_best = pl->d_best;
    w.pair_score = pl->d_score;
    w.rec = pl->d_rec;
    w.heads = pl->d_heads;
    w.timing = timing;
    w.gap = pl->gap;
    w.key_rowbits = pl->key_rowbits;
    w.fast = kn.tb_generic ? 0 : 1;
    w.stager = kn.tb_stager ? 1 : 0;
    w.text = pl->d_text_in;
    w.pattern = pl->d_pattern_in;
    w.score_tab = pl->d_table;
    w.A = pl->A;
    w.tb_pg = nullptr;
    w.cap = kn.tb_cap;
    if (!pl->tb_groups.empty())
    {
        // table traceback; its last kernel walks the pairs the tables leave, so the sequential walk
        // runs only when some pair has no groups
        TbArgs t;
        t.strips = pl->d_strips;
        t.pairs = pl->d_pairs;
        t.masks = pl->d_masks;
        t.groups = pl->d_tbgroups;
        t.pair_g0 = pl->d_tbpg;
        t.pair_score = pl->d_score;
        t.strip_best = pl->d_best;
        t.start = pl->d_tbstart;
        t.sent = pl->d_sent;
        t.sdelta = pl->d_sdelta;
        t.send = pl->d_send;
        t.pend = pl->d_pend;
        t.text = pl->d_text_in;
        t.pattern = pl->d_pattern_in;
        t.score_tab = pl->d_table;
        t.A = pl->A;
        t.gap = pl->gap;
        t.key_rowbits = pl->key_rowbits;
        t.local = pl->mode == SA_LOCAL ? 1 : 0;
        t.dbg = nullptr;
        DevPtr<uint64_t> dbgBuf;
        const size_t dbgWords = 12 * pl->strips.size();
        if (kn.tb_table_timing)
        {
            HIP_TRY(hipMalloc((void **)&t.dbg, sizeof(uint64_t) * dbgWords));
            dbgBuf.reset(t.dbg);
            HIP_TRY(hipMemsetAsync(t.dbg, 0, sizeof(uint64_t) * dbgWords, st));
        }
        t.tbl = pl->d_tbl;
        t.win = pl->d_win;
        t.gtbl = pl->d_gtbl;
        t.gent = pl->d_gent;
        t.tb_flag = pl->d_tbflag;
        t.rec = pl->d_rec;
        t.heads = pl->d_heads;
        t.fast = w.fast;
        // rounds of tables: pairs past 131072 rows stray further from the first round's line than its
        // windows reach (random DNA: 800 columns at 120000^2, 3000 at 250000^2; tools/path_deviation.py);
        // a round with nothing pending costs its three launches
        const int rounds = kn.tb_rounds > 0 ? kn.tb_rounds : (pl->max_recs > 131072 ? 8 : 1);
        t.strict = kn.tb_strict ? 1 : 0;
        t.round = 1;
        w.tb_pg = pl->d_tbpg;
        // strip tables of 1024 threads when every strip has a CU of its own (SA_TB_WIDE=0: always 512)
        const bool wide = knobs().tb_wide && (int)pl->strips.size() <= pl->num_cu;
        launch_tb(t, w, (int)pl->strips.size(), (int)pl->tb_groups.size(), np, rounds, wide, st);
        HIP_TRY(hipGetLastError());
        if (kn.tb_table_timing)
        {
            std::vector<uint64_t> v(dbgWords);
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipMemcpy(v.data(), t.dbg, v.size() * 8, hipMemcpyDeviceToHost));
            if (FILE *f = std::fopen(kn.tb_table_timing, "wb"))
            {
                std::fwrite(v.data(), 8, v.size(), f);
                std::fclose(f);
            }
        }
        if (int rc = debug_sync(st, "table traceback")) return rc;
    }
    bool sequential = pl->tb_groups.empty();
    for (int64_t p = 0; p < np && !sequential; ++p) sequential = pl->tb_pg[p + 1] == pl->tb_pg[p];
    if (sequential) launch_walk(pl->R, pl->mode == SA_LOCAL, w, np, st);
    HIP_TRY(hipGetLastError());
    if (int rc = debug_sync(st, "walk kernel")) return rc;
    ExpandArgs x;
    x.text = pl->d_text_in;
    x.pattern = pl->d_pattern_in;
    x.pairs = pl->d_pairs;
    x.rec = pl->d_rec;
    x.heads = pl->d_heads;
    x.out_text = pl->d_out_text;
    x.out_pattern = pl->d_out_pattern;
    x.results = pl->d_results;
    x.ctrl = pl->d_ctrl;
    x.A = pl->A;
    std::memcpy(x.alphabet, pl->alphabet, 33);
    x.chunk_sums = pl->d_csum;
    x.chunk_flags = pl->d_cflag;
    x.epoch = pl->epoch;
    // records per pair: one per row (row walk, R = 1) or per column (column walk)
    launch_expand(x, np, pl->max_recs, st);
    HIP_TRY(hipGetLastError());
    if (int rc = debug_sync(st, "expand_kernel")) return rc;
    if (tmPath)
    {
        std::vector<uint64_t> tm(9 * (size_t)np);
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpy(tm.data(), timing, tm.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = std::fopen(tmPath, "wb"))
        {
            std::fwrite(tm.data(), 8, tm.size(), f);
            std::fclose(f);
        }
    }
    return SA_OK;
}

int sa_plan_fetch_results(sa_plan *pl, sa_result *out, void *stream)
{
    if (!pl || !out) return fail(SA_ERR_INVALID, "sa_plan_fetch_results: null argument");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    Control ctrl;
    HIP_TRY(hipMemcpyAsync(&ctrl, pl->d_ctrl, sizeof(Control), hipMemcpyDeviceToHost, st));
    if (out && !pl->pairs.empty())
        HIP_TRY(hipMemcpyAsync(out, pl->d_results, sizeof(sa_result) * pl->pairs.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (ctrl.bad_input == pl->epoch) return fail(SA_ERR_INVALID, "a text or pattern byte is outside the alphabet (0..A-1)");
    if (ctrl.abort_flag) return fail(SA_ERR_TIMEOUT, "fill aborted: a strip hand-off timed out");
    return SA_OK;
}

int sa_plan_fetch_alignment(sa_plan *pl, int64_t index, char *at, char *ap, uint64_t cap, void *stream)
{
    if (!pl || index < 0 || index >= (int64_t)pl->pairs.size()) return fail(SA_ERR_INVALID, "sa_plan_fetch_alignment: bad index");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    sa_result r;
    HIP_TRY(hipMemcpyAsync(&r, pl->d_results + index, sizeof(r), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (r.num_alignment_bytes > cap) return fail(SA_ERR_INVALID, "output capacity too small");
    const uint64_t off = pl->pairs[index].out_off;
    if (r.num_alignment_bytes)
    {
        if (at) HIP_TRY(hipMemcpyAsync(at, pl->d_out_text + off, r.num_alignment_bytes, hipMemcpyDeviceToHost, st));
        if (ap) HIP_TRY(hipMemcpyAsync(ap, pl->d_out_pattern + off, r.num_alignment_bytes, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return SA_OK;
}

uint64_t sa_plan_output_bytes(const sa_plan *pl) { return pl ? pl->out_bytes : 0; }

int sa_plan_fetch_all(sa_plan *pl, sa_result *out, char *tb, char *pb, uint64_t buf_bytes, uint64_t *offsets,
                      void *stream)
{
    if (!pl || (!pl->pairs.empty() && !offsets)) return fail(SA_ERR_INVALID, "sa_plan_fetch_all: null argument");
    if ((tb || pb) && buf_bytes < pl->out_bytes) return fail(SA_ERR_INVALID, "sa_plan_fetch_all: buffers below sa_plan_output_bytes");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    Control ctrl;
    HIP_TRY(hipMemcpyAsync(&ctrl, pl->d_ctrl, sizeof(Control), hipMemcpyDeviceToHost, st));
    if (out && !pl->pairs.empty())
        HIP_TRY(hipMemcpyAsync(out, pl->d_results, sizeof(sa_result) * pl->pairs.size(), hipMemcpyDeviceToHost, st));
    if (tb && pl->out_bytes) HIP_TRY(hipMemcpyAsync(tb, pl->d_out_text, pl->out_bytes, hipMemcpyDeviceToHost, st));
    if (pb && pl->out_bytes) HIP_TRY(hipMemcpyAsync(pb, pl->d_out_pattern, pl->out_bytes, hipMemcpyDeviceToHost, st));
    for (size_t i = 0; i < pl->pairs.size(); ++i) offsets[i] = pl->pairs[i].out_off;
    HIP_TRY(hipStreamSynchronize(st));
    if (ctrl.bad_input == pl->epoch) return fail(SA_ERR_INVALID, "a text or pattern byte is outside the alphabet (0..A-1)");
    if (ctrl.abort_flag) return fail(SA_ERR_TIMEOUT, "fill aborted: a strip hand-off timed out");
    return SA_OK;
}

int sa_plan_fetch_directions(sa_plan *pl, int64_t index, uint8_t *M, void *stream)
{
    if (!pl || !M || index < 0 || index >= (int64_t)pl->pairs.size()) return fail(SA_ERR_INVALID, "sa_plan_fetch_directions: bad argument");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    const PairDesc &pd = pl->pairs[index];
    const uint64_t n = pd.text_len, m = pd.pattern_len, cols = n + 1;
    const bool local = pl->mode == SA_LOCAL;
    for (uint64_t j = 0; j < cols; ++j) M[j] = local ? 3 : 0;          // row 0: STOP / LEFT
    for (uint64_t i = 1; i <= m; ++i) M[i * cols] = local ? 3 : 2;     // column 0: STOP / TOP
    if (pd.num_strips == 0) return SA_OK;
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    const StripDesc &first = pl->strips[pd.first_strip];
    const StripDesc &last = pl->strips[pd.first_strip + pd.num_strips - 1];
    const uint64_t e0 = first.mask_off, e1 = last.mask_off + (uint64_t)last.nsteps * pl->R;
    std::vector<uint32_t> h((e1 - e0) * 4);
    HIP_TRY(hipMemcpyAsync(h.data(), pl->d_masks + e0 * 4, h.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int R = pl->R, RB = kWave * R;
    const uint64_t CS = std::max(32, pl->U * R), NW = CS / 32, LW = 2 * NW;  // Cfg<R>
    for (uint64_t i = 1; i <= m; ++i)
    {
        const uint64_t b = (i - 1) / RB, il = (i - 1) % RB, k = il / R, rho = il % R;
        const StripDesc &sd = pl->strips[pd.first_strip + b];
        for (uint64_t j = 1; j <= n; ++j)
        {
            // slot e of the strip: chunk e/CS, lane k's LW words; R = 1: interleaved word (e%32)/16,
            // bits 31 - 2(e%16) / 30 - 2(e%16); R > 1: plane word (e%CS)/32, bit 31-e%32
            const uint64_t e = (j - 1 + k) * R + rho;
            const uint32_t *w = &h[(sd.mask_off - e0) * 4 + (e / CS) * kWave * LW + k * LW];
            uint32_t b0, b1;
            if (R == 1)
            {
                const uint32_t x = w[(e % 32) / 16];
                b0 = (x >> (31 - 2 * (e % 16))) & 1u;
                b1 = (x >> (30 - 2 * (e % 16))) & 1u;
            }
            else
            {
                b0 = (w[(e % CS) / 32] >> (31 - e % 32)) & 1u;
                b1 = (w[NW + (e % CS) / 32] >> (31 - e % 32)) & 1u;
            }
            // global: plane1 is the raw "up > left" bit and DIAG wins (see run_body)
            // global, and local R = 1 (raw decisions, no STOP: sa_layout.h): DIAG wins over the raw
            // "up > left"; local R > 1: the plane pair is the reference's code itself
            M[i * cols + j] = (uint8_t)(pl->mode == SA_GLOBAL || R == 1 ? (b0 ? 1u : (b1 ? 2u : 0u)) : (b0 | (b1 << 1)));
        }
    }
    if (local && R == 1)
    {
        // local R = 1 planes hold the raw decisions (the walk recovers STOP from H along the path):
        // the reference's M has STOP wherever best <= 0, i.e. H == 0 (alignSequenceCPU.cpp:175-190),
        // so H is recomputed here row by row from the fill's inputs and those cells are overwritten
        if (!pl->filled || !pl->d_text_in || !pl->d_pattern_in)
            return fail(SA_ERR_INVALID, "sa_plan_fetch_directions: the plan has not been filled");
        std::vector<int8_t> tx(n), px(m);
        HIP_TRY(hipMemcpyAsync(tx.data(), pl->d_text_in + pd.text_off, n, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(px.data(), pl->d_pattern_in + pd.pattern_off, m, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int8_t c : tx)
            if (c < 0 || c >= pl->A) return fail(SA_ERR_INVALID, "sa_plan_fetch_directions: text letter outside the alphabet");
        for (int8_t c : px)
            if (c < 0 || c >= pl->A) return fail(SA_ERR_INVALID, "sa_plan_fetch_directions: pattern letter outside the alphabet");
        const int64_t g = pl->gap;
        std::vector<int64_t> prev(cols, 0), cur(cols, 0);
        for (uint64_t i = 1; i <= m; ++i)
        {
            cur[0] = 0;
            const int32_t *srow = &pl->h_table[(size_t)px[i - 1] * pl->A];  // S + g (local table)
            for (uint64_t j = 1; j <= n; ++j)
            {
                const int64_t d = prev[j - 1] + srow[tx[j - 1]] - g, l = cur[j - 1] - g, u = prev[j] - g;
                const int64_t best = std::max(d, std::max(l, u));
                cur[j] = best > 0 ? best : 0;
                if (best <= 0) M[i * cols + j] = 3;
            }
            std::swap(prev, cur);
        }
    }
    return SA_OK;
}

int sa_plan_info(const sa_plan *pl, int64_t *num_strips, int32_t *rows_per_lane, uint64_t *device_bytes,
                 uint64_t *mask_bytes)
{
    if (!pl) return fail(SA_ERR_INVALID, "sa_plan_info: null plan");
    if (num_strips) *num_strips = (int64_t)pl->strips.size();
    if (rows_per_lane) *rows_per_lane = pl->R;
    if (device_bytes) *device_bytes = pl->bytes_total;
    if (mask_bytes) *mask_bytes = pl->bytes_masks;
    return SA_OK;
}

int sa_plan_fill_kind(const sa_plan *pl)
{
    if (!pl) return fail(SA_ERR_INVALID, "sa_plan_fill_kind: null plan");
    if (pl->sk == kPair) return pl->chain ? SA_FILL_PAIR_CHAIN : SA_FILL_PAIR;
    return pl->band ? SA_FILL_BAND : SA_FILL_STRIPS;
}

const void *sa_plan_device_results(const sa_plan *pl) { return pl ? (const void *)pl->d_results : nullptr; }

int sa_plan_copy_results(const sa_plan *pl, void *d_dst, void *stream)
{
    if (!pl || (!d_dst && !pl->pairs.empty())) return fail(SA_ERR_INVALID, "sa_plan_copy_results: null argument");
    if (pl->pairs.empty()) return SA_OK;
    DeviceGuard dg(pl->device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    HIP_TRY(hipMemcpyAsync(d_dst, pl->d_results, sizeof(sa_result) * pl->pairs.size(), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
    return SA_OK;
}

int sa_align_pair(const sa_params *P, const char *text, uint64_t n, const char *pattern, uint64_t m, int device,
                  sa_result *out, char *at, char *ap, uint64_t cap, double *fill_us)
{
    if (!P || !out || (n && !text) || (m && !pattern)) return fail(SA_ERR_INVALID, "sa_align_pair: null argument");
    const bool fillOnly = !at && !ap;  // -DBENCHMARK contract: DP fill only
    if (!fillOnly && cap < n + m) return fail(SA_ERR_INVALID, "sa_align_pair: output capacity below text_len + pattern_len");
    // (letters outside the alphabet are reported by the encode kernel: SA_ERR_INVALID below)
    DeviceCtx *ws = device_ctx(device);
    if (!ws) return fail(SA_ERR_INVALID, "sa_align_pair: bad device");
    std::lock_guard<std::mutex> lk(ws->mu);
    DeviceGuard dg(device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    // the plan, its uploads and both inputs live in the device's cached arena: one copy up (plan
    // creation), one copy down (control word, result, strings) and the kernels in between
    sa_pair pr{0, n, 0, m};
    OneShotInputs in;
    in.text = text;
    in.n = n;
    in.pattern = pattern;
    in.m = m;
    sa_plan *pl = nullptr;
    int rc = plan_create(P, &pr, 1, device, ws, &in, &pl);
    if (rc) return rc;
    std::unique_ptr<sa_plan, void (*)(sa_plan *)> hold(pl, free_plan);
    HIP_TRY(hipSetDevice(device));
    hipStream_t st = ws->stream;
    HIP_TRY(hipEventRecord(ws->e0, st));
    if ((rc = sa_plan_fill(pl, pl->d_ws_text, pl->d_ws_pattern, st))) return rc;
    HIP_TRY(hipEventRecord(ws->e1, st));
    if (!fillOnly && (rc = sa_plan_traceback(pl, st))) return rc;
    // [ctrl | result | out_text | out_pattern]; fill-only needs the control word alone
    const size_t dn = fillOnly ? sizeof(Control) : pl->dn_bytes;
    if (knobs().stage_kernel) HIP_TRY(stage_copy(ws->pinned_dev, pl->d_dn, dn, st));
    else HIP_TRY(hipMemcpyAsync(ws->pinned, pl->d_dn, dn, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const char *h = ws->pinned;
    Control ctrl;
    std::memcpy(&ctrl, h, sizeof(Control));
    // also in fill-only mode: a fill whose hand-off timed out produced garbage, not a fill time
    if (ctrl.bad_input == pl->epoch) return fail(SA_ERR_INVALID, "a text or pattern byte is outside the alphabet (0..A-1)");
    if (ctrl.abort_flag) return fail(SA_ERR_TIMEOUT, "fill aborted: a strip hand-off timed out");
    if (!fillOnly)
    {
        std::memcpy(out, h + ((char *)pl->d_results - pl->d_dn), sizeof(sa_result));
        const uint64_t L = std::min<uint64_t>(out->num_alignment_bytes, n + m);
        const uint64_t off = pl->pairs[0].out_off;
        if (at && L) std::memcpy(at, h + ((char *)pl->d_out_text - pl->d_dn) + off, L);
        if (ap && L) std::memcpy(ap, h + ((char *)pl->d_out_pattern - pl->d_dn) + off, L);
    }
    if (fill_us)
    {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, ws->e0, ws->e1));
        *fill_us = 1000.0 * ms;
    }
    return SA_OK;
}

int sa_release_workspace(int device)
{
    std::vector<DeviceCtx *> v;
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        v = g_ctx;
    }
    for (int d = 0; d < (int)v.size(); ++d)
        if (v[d] && (device < 0 || device == d)) release_ctx(v[d]);
    return SA_OK;
}

int sa_selftest(int device)
{
    DeviceGuard dg(device);
    if (!dg.ok) return fail(SA_ERR_HIP, "hipSetDevice failed");
    int *d = nullptr;
    HIP_TRY(hipMalloc(&d, 6 * 64 * sizeof(int)));
    hipLaunchKernelGGL(selftest_kernel, dim3(1), dim3(64), 0, 0, d);
    std::vector<int> h(6 * 64);
    HIP_TRY(hipMemcpy(h.data(), d, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(d));
    uint64_t b = 0;
    for (int l = 0; l < 64; ++l)
        if (l % 3 == 0) b |= 1ull << l;
    const int sbfe[4] = {5, 10, -9, 24};
    for (int l = 0; l < 64; ++l)
    {
        if (h[l] != (l == 0 ? -1 : 100 + l - 1)) return fail(SA_ERR_UNSUPPORTED, "DPP wave_shr:1 mismatch at lane " + std::to_string(l));
        if (h[64 + l] != (l == 63 ? -2 : 100 + l + 1)) return fail(SA_ERR_UNSUPPORTED, "DPP wave_shl:1 mismatch at lane " + std::to_string(l));
        if (h[128 + l] != 100 + (l + 1) % 64) return fail(SA_ERR_UNSUPPORTED, "DPP wave_rol:1 mismatch at lane " + std::to_string(l));
        const int wl = l == 5 ? (int)(uint32_t)b : (l == 6 ? (int)(uint32_t)(b >> 32) : 0);
        if (h[192 + l] != wl) return fail(SA_ERR_UNSUPPORTED, "ballot/writelane mismatch at lane " + std::to_string(l));
        if (h[256 + l] != sbfe[l & 3]) return fail(SA_ERR_UNSUPPORTED, "v_bfe_i32 mismatch at lane " + std::to_string(l));
        if (h[320 + l] <= 0) return fail(SA_ERR_UNSUPPORTED, "s_memrealtime does not advance (" + std::to_string(h[320 + l]) + ")");
    }
    return SA_OK;
}

}  // extern "C"
