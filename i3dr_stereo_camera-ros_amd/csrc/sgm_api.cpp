// sgm_api.cpp — C-ABI of libsgm_hip.so (include/sgm_hip.h).
//
// The handle owns one HIP stream and one device workspace on its device. Geometry-
// dependent buffers are (re)allocated lazily at the first match and whenever W, H, D or
// the mode change — mirroring the reference, which constructs its matchers lazily at the
// first frame (generate_disparity.cpp:342-346) and never frees them.
// A per-handle mutex serialises set_params against match (the reference's only locking
// matcher does the same: I3DRSGM.cpp:152, :635).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sgm_device.h"
#include "sgm_hip.h"

namespace sgm {
hipError_t launch_census(const uint8_t*, const uint8_t*, size_t, int, int, uint64_t*, uint64_t*, hipStream_t);
int census_path_items(const Geom&, unsigned, int, int, uint32_t*, int, int up_group = 0);
hipError_t launch_census_paths(const PathFrames&, size_t, const Geom&, const uint32_t*, int, hipStream_t,
                               const uint8_t* = nullptr, const uint8_t* = nullptr, size_t = 0);
hipError_t launch_census_wta(const WtaFrames&, size_t, const Geom&, size_t, hipStream_t);
hipError_t launch_rectify_map(const double*, const double*, const double*, int, int, float*, float*, size_t,
                              hipStream_t);
hipError_t launch_remap_cubic(const uint8_t*, size_t, int, int, const float*, const float*, size_t, int, int,
                              const int16_t*, uint8_t*, size_t, hipStream_t);
void cubic_table(int16_t*);
bool rectify_inverse(const double*, const double*, double*);
hipError_t launch_census_tiles(const CensusFrames&, int, int, hipStream_t);
hipError_t launch_census_fused(const PathFrames&, const WtaFrames&, const CensusFrames&, size_t, const Geom&,
                               const uint32_t*, int, size_t, bool, hipStream_t);
hipError_t launch_census_rowfin(const WtaFrames&, const Geom&, size_t, hipStream_t);
hipError_t launch_median3(const int16_t*, size_t, int16_t*, size_t, int, int, hipStream_t);
hipError_t launch_speckle(const int16_t*, size_t, int16_t*, size_t, int, int, int, int, int, int*, int*, hipStream_t);
hipError_t launch_fill16(int16_t*, size_t, int, int, int, hipStream_t);
hipError_t launch_to_f32(const int16_t*, size_t, float*, size_t, int, int, hipStream_t);
hipError_t launch_disp_to_msg(const int16_t*, size_t, int, int, float, float, float*, size_t, hipStream_t);
hipError_t launch_depth_points(const float*, size_t, int, int, const float*, double, double, const uint8_t*, size_t,
                               int, float*, size_t, float4*, int, int*, int*, hipStream_t);
hipError_t launch_ocv_cost(const uint8_t*, const uint8_t*, size_t, const Geom&, int, uint8_t*, int16_t*, int16_t*,
                           hipStream_t);
bool ocv_cost_takes_fused(const Geom&);
hipError_t launch_ocv_paths(const int16_t*, const int16_t*, void*, size_t, const Geom&, int, hipStream_t,
                            int skipdir = -1);
hipError_t launch_ocv_vwta(const int16_t*, const int16_t*, const void*, size_t, int, const Geom&, uint64_t*, hipStream_t);
int ocv_vwta_dir(int ndir);
hipError_t launch_ocv_wta(const int16_t*, const void*, size_t, int, const Geom&, int16_t*, size_t, hipStream_t);
int ocv_evol_mode(const Geom&, int, int);
}  // namespace sgm

using sgm::Geom;

// measurement-only build knobs (tools/build_variant.sh ... sgm_api.cpp)
#ifndef SGM_VOL_PAD_BYTES
#define SGM_VOL_PAD_BYTES 0    // extra bytes per census volume slot
#endif
#ifndef SGM_IO_PRIO
#define SGM_IO_PRIO 1          // host-I/O copy streams at the highest stream priority
#endif

namespace {

constexpr size_t kAlign = 256;
constexpr size_t kTrashBytes = 4096;   // >= 64 lanes x 32 disparities (census_sgm.hip trash stores)
inline size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

// effective parameters — identical rules to the oracle (oracle/sgm_oracle.c effective())
int make_geom(const sgm_params& p, int W, int H, Geom& g, std::string& err)
{
    if (W <= 0 || H <= 0) { err = "image size must be positive"; return SGM_ERR_ARG; }
    if (W > 32767 || H > 32767) { err = "image larger than 32767 pixels"; return SGM_ERR_UNSUPPORTED; }
    if (p.mode < SGM_MODE_OCV_SGBM5 || p.mode > SGM_MODE_CENSUS8) { err = "unknown mode"; return SGM_ERR_PARAM; }
    if (p.num_disparities <= 0 || p.num_disparities % 16 != 0) {
        err = "numDisparities must be a positive multiple of 16 (OpenCV: CV_Assert(D % 16 == 0))";
        return SGM_ERR_PARAM;
    }
    // OCV modes: up to 2048 (the node's cfg range, i3DR_Disparity.cfg:27); census mode: 512
    // (its u8 path engine keeps at most 32 disparities per lane of a 16-lane line)
    const int max_d = p.mode == SGM_MODE_CENSUS8 ? 512 : 2048;
    if (p.num_disparities > max_d) {
        err = p.mode == SGM_MODE_CENSUS8 ? "numDisparities > 512 is not supported in the census mode"
                                         : "numDisparities > 2048 is not supported";
        return SGM_ERR_UNSUPPORTED;
    }
    g = Geom{};
    g.W = W; g.H = H;
    g.minD = p.min_disparity; g.D = p.num_disparities;
    const int maxD = g.minD + g.D;
    if (p.mode == SGM_MODE_CENSUS8) {
        g.P1 = p.p1 > 0 ? p.p1 : 10;
        g.P2 = std::max(p.p2 > 0 ? p.p2 : 120, g.P1 + 1);
        if (g.P2 > 193) g.P2 = 193;                   // u8 path costs: 62 + P2 <= 255
        if (g.P1 >= g.P2) g.P1 = g.P2 - 1;
        g.subpix = p.subpixel != 0; g.lr = p.lr_check != 0;
        g.SW2 = 4; g.SH2 = 3; g.ftzero = 0;
    } else {
        const int sw = p.block_size > 0 ? p.block_size : 5;
        g.SW2 = sw / 2; g.SH2 = sw / 2;
        g.ftzero = std::max(p.prefilter_cap, 15) | 1;
        g.P1 = p.p1 > 0 ? p.p1 : 2;
        g.P2 = std::max(p.p2 > 0 ? p.p2 : 5, g.P1 + 1);
        g.subpix = 1; g.lr = 1;
        // A pixel cost is <= 2*ftzero + 63 (BT of the prefiltered image + raw BT >> 2), so
        // C = box sum + P2 stays in int16 below this bound, and then every path cost lies in
        // [C - P2, C]: int16 volumes are exact. Above it C may wrap (OpenCV's CostType) and a
        // path cost can leave int16, while OpenCV adds the int value into S: int32 volumes.
        // When the bound allows it, the cost kernel flags the C' values that do leave int16 and
        // only frames with such a value take the int32 volumes (Geom::wide == 2): real images
        // stay far below the bound (the reference launch config, block 21: bound 41 413).
        // SGM_OCV_WIDE=1 forces int32 volumes; SGM_OCV_GATE=0 takes them whenever the bound allows.
        // The SIMD branches (ocv_compat SGM_OCV_SIMD_SAT) saturate instead, and agree with the
        // plain kernels until a C' exceeds 32767 - P2 (then (short)(minLr + P2) can wrap): their
        // flagged kernels are the sequential saturating cost and saturating int16 paths / sums.
        g.compat = p.ocv_compat & (SGM_OCV_COL0_LEGACY | SGM_OCV_SIMD_SAT | SGM_OCV_LANE_TIE);
        const bool sat = (g.compat & SGM_OCV_SIMD_SAT) != 0;
        g.ovf_thr = sat ? 32767 - g.P2 : 32767;
        const long long cmax = (long long)(2 * g.SW2 + 1) * (2 * g.SH2 + 1) * (2 * g.ftzero + 63) + g.P2 +
                               (sat ? g.P2 : 0);
        const char* wide_env = std::getenv("SGM_OCV_WIDE");
        const char* gate_env = std::getenv("SGM_OCV_GATE");
        if (wide_env && std::atoi(wide_env) != 0) g.wide = 1;
        else if (cmax > 32767) g.wide = (gate_env && std::atoi(gate_env) == 0) ? 1 : 2;
        else g.wide = 0;
    }
    g.uniq = p.uniqueness_ratio >= 0 ? p.uniqueness_ratio : 10;
    g.disp12 = p.disp12_max_diff > 0 ? p.disp12_max_diff : 1;
    g.minX1 = std::max(maxD, 0);
    g.maxX1 = W + std::min(g.minD, 0);
    g.width1 = g.maxX1 - g.minX1;
    g.invalid = (g.minD - 1) * 16;
    return SGM_OK;
}

bool use_median(const sgm_params& p) { return p.mode != SGM_MODE_CENSUS8 || p.median != 0; }

struct Workspace {
    void* base = nullptr;
    size_t size = 0;
};

}  // namespace

struct sgm_handle {
    int device = 0;
    sgm_params params{};
    hipStream_t stream = nullptr;
    std::string err;
    std::mutex mu;
    Workspace ws;
    uint8_t* pin = nullptr;      // pinned host staging
    size_t pin_size = 0;
    // profiling: one hipEvent before every launch and one after the last launch of a
    // match; launch k runs from event `start` to the next recorded event
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;   // grows on demand, reused after a re-enable
    size_t ev_used = 0;
    struct LaunchRec { int stage; size_t ev0, ev1; };
    std::vector<LaunchRec> launches;
    int prof_frames = 0;
    int nstages = 0;                   // distinct stage names seen (first-launch order)
    const char* stage_name[SGM_MAX_STAGES] = {};
    double stage_bytes[SGM_MAX_STAGES] = {};
    std::vector<sgm_handle*> sub;  // per-device handles for sgm_match_batch
    int n_cu = 0;                  // compute units of the device (path work-list dealing)
    int* aux = nullptr;            // per-row counts / offsets of sgm_depth_points
    size_t aux_n = 0;
    uint32_t* items_pin = nullptr; // pinned host copy of the uploaded path work list
    int items_cap = 0;
    std::string items_key[2];      // geometry + workspace each device copy (single / group) belongs to
    int16_t* cubic_tab = nullptr;  // device INTER_CUBIC weight table (sgm_remap_cubic), built once
    bool rect_on = false;          // sgm_set_rectification: batch inputs are raw, rectified in the census
    sgm::RectifyIn rect{};
    // exact tile mode (sgm_match_tiled_exact): one handle per row band, each with a second
    // stream for its upward sweeps and four events (census, down, up, gather)
    std::vector<sgm_handle*> bands;
    // OCV-mode frame batches: frames dealt over a few same-device handles, each with its own
    // stream and workspace, so the small launches of one frame overlap another's
    std::vector<sgm_handle*> par;
    hipEvent_t par_ev = nullptr;   // recorded on the handle's stream, then each lane's done
    hipStream_t stream2 = nullptr;
    hipEvent_t bev[4] = {};
    // cross-call ordering: every call that uses the workspace records `done` on the stream it
    // ran on, and the next call (whatever its stream) waits on it first
    hipEvent_t done = nullptr;
    hipStream_t done_stream = nullptr;
    // host-buffer frame streaming (sgm_match_batch): device + pinned rings, copy streams
    void* io_dev = nullptr;
    size_t io_dev_size = 0;
    uint8_t* io_pin = nullptr;
    size_t io_pin_size = 0;
    hipStream_t up = nullptr, down = nullptr;
    std::vector<hipEvent_t> io_ev;
    // host buffers page-locked and mapped by sgm_host_register (host range -> device address)
    struct HostReg { char* host; size_t bytes; char* dev; };
    std::vector<HostReg> regs;
    // host-buffer matches: the right image's copy runs on `cpy` beside the left image's census
    hipStream_t cpy = nullptr;
    hipEvent_t cpy_ev = nullptr;
};

namespace {

int fail(sgm_handle* h, int code, const std::string& msg)
{
    if (h) h->err = msg;
    return code;
}

int hip_fail(sgm_handle* h, hipError_t e, const char* where)
{
    return fail(h, SGM_ERR_DEVICE, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, where)                                   \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) return hip_fail(h, e_, where);   \
    } while (0)

int ensure_stream(sgm_handle* h)
{
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    if (!h->stream) HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking), "hipStreamCreate");
    if (!h->done) HIP_TRY(hipEventCreateWithFlags(&h->done, hipEventDisableTiming), "hipEventCreate");
    if (!h->n_cu) HIP_TRY(hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, h->device), "attr");
    return SGM_OK;
}

// Orders a call on stream `st` after the previous call that used the handle's workspace
// (on any stream): the workspace (codes, volumes, scratch) is shared by all calls.
int order_after_last(sgm_handle* h, hipStream_t st)
{
    if (h->done_stream && h->done_stream != st) HIP_TRY(hipStreamWaitEvent(st, h->done, 0), "hipStreamWaitEvent");
    return SGM_OK;
}

// Marks the end of a call's work on `st` (see order_after_last).
int mark_done(sgm_handle* h, hipStream_t st)
{
    HIP_TRY(hipEventRecord(h->done, st), "hipEventRecord");
    h->done_stream = st;
    return SGM_OK;
}

// Records the next pool event on the handle's stream; returns its index or -1.
long record_event(sgm_handle* h)
{
    if (h->ev_used == h->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return -1;
        h->ev_pool.push_back(e);
    }
    if (hipEventRecord(h->ev_pool[h->ev_used], h->stream) != hipSuccess) return -1;
    return (long)h->ev_used++;
}

int stage_index(sgm_handle* h, const char* name, double bytes)
{
    for (int i = 0; i < h->nstages; i++)
        if (std::strcmp(h->stage_name[i], name) == 0) { h->stage_bytes[i] = bytes; return i; }
    if (h->nstages == SGM_MAX_STAGES) return -1;
    h->stage_name[h->nstages] = name;
    h->stage_bytes[h->nstages] = bytes;
    return h->nstages++;
}

int ensure_ws(sgm_handle* h, size_t bytes)
{
    if (h->ws.size >= bytes) return SGM_OK;
    h->items_key[0].clear();       // contents (the path work lists) do not survive
    h->items_key[1].clear();
    if (h->ws.base) {
        (void)hipStreamSynchronize(h->stream);
        if (h->done_stream) (void)hipEventSynchronize(h->done);
        (void)hipFree(h->ws.base);
        h->ws.base = nullptr;
        h->ws.size = 0;
    }
    hipError_t e = hipMalloc(&h->ws.base, bytes);
    if (e != hipSuccess) {
        h->ws.base = nullptr;
        return fail(h, SGM_ERR_ALLOC, std::string("hipMalloc workspace: ") + hipGetErrorString(e));
    }
    h->ws.size = bytes;
    return SGM_OK;
}

int ensure_pin(sgm_handle* h, size_t bytes)
{
    if (h->pin_size >= bytes) return SGM_OK;
    if (h->pin) { (void)hipStreamSynchronize(h->stream); (void)hipHostFree(h->pin); h->pin = nullptr; h->pin_size = 0; }
    hipError_t e = hipHostMalloc((void**)&h->pin, bytes, hipHostMallocDefault);
    if (e != hipSuccess) { h->pin = nullptr; return fail(h, SGM_ERR_ALLOC, "hipHostMalloc staging"); }
    h->pin_size = bytes;
    return SGM_OK;
}

// The INTER_CUBIC weight table on the device, built on the host once per handle.
int ensure_cubic_table(sgm_handle* h)
{
    if (h->cubic_tab) return SGM_OK;
    std::vector<int16_t> tab(32 * 32 * 16);
    sgm::cubic_table(tab.data());
    int16_t* d = nullptr;
    hipError_t e = hipMalloc(&d, tab.size() * 2);
    if (e != hipSuccess) return hip_fail(h, e, "hipMalloc cubic table");
    e = hipMemcpy(d, tab.data(), tab.size() * 2, hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(d); return hip_fail(h, e, "upload cubic table"); }
    h->cubic_tab = d;
    return SGM_OK;
}

// Workspace carve-up for one geometry. Offsets are 256-B aligned.
struct Layout {
    // census: set 0 serves single matches; a pipelined batch uses code sets 0 .. 3*group-1
    // (the census of group k+1 runs beside the up+WTA sweeps of group k-1), volume sets
    // 0 .. 2*group-1 and one up+WTA result image per frame of a group
    size_t cL[3 * sgm::kMaxGroup] = {}, cR[3 * sgm::kMaxGroup] = {}, vols[2 * sgm::kMaxGroup] = {};
    size_t res[sgm::kMaxGroup] = {};
    size_t vol_bytes = 0;
    int group = 1;                                         // frames per pipelined launch
    bool up_wta = false;                                   // pipelined batch: up+WTA scheme
    size_t items[2] = {}; int n_items[2] = {};             // path work lists: one frame / a group
    size_t planes = 0, bufA = 0, bufB = 0, ovols = 0, ovf = 0;  // ocv
    size_t ores = 0;                                       // ocv: per-pixel results of k_ocv_vwta
    size_t tmp = 0, lab = 0, cnt = 0;                      // post
    size_t inL = 0, inR = 0, out = 0, outf = 0;            // host-API staging (int16 / float out)
    size_t total = 0;
};

// Pipelined census batches with D <= 256 fuse the upward vertical sweep with the WTA
// (census_sgm.hip UpWta) unless SGM_UPWTA=0 (the earlier scheme: 8 volumes written, WTA rows
// interleaved).
bool use_up_wta()
{
    const char* e = std::getenv("SGM_UPWTA");
    return !e || std::atoi(e) != 0;
}

Layout make_layout(const sgm_params& p, const Geom& g, bool host_io, int group = 0)
{
    Layout l;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + std::max<size_t>(bytes, 1)); return o; };
    auto take_codes = [&](size_t n) { return take((n + 2 * sgm::kCodeMargin) * 8) + 8 * sgm::kCodeMargin; };
    const size_t WH = (size_t)g.W * g.H;
    const size_t cells = (size_t)std::max(g.width1, 0) * g.H * g.D;
    if (p.mode == SGM_MODE_CENSUS8) {
        l.vol_bytes = align_up(cells + kTrashBytes);   // + trash slot for masked stores
#if SGM_VOL_PAD_BYTES > 0
        // extra bytes per volume slot (a measurement build: tools/build_variant.sh, -DSGM_VOL_PAD_BYTES=N)
        l.vol_bytes = align_up(l.vol_bytes + (size_t)std::min<long long>(SGM_VOL_PAD_BYTES, 1LL << 30));
#endif
        l.group = std::max(group, 1);
        // D > 256 (32 disparities per lane, 2 waves/SIMD) keeps the earlier scheme: its up+WTA
        // blocks are long latency-bound chains (C5 batch: 32.3 vs 23.3 ms per frame)
        l.up_wta = group > 0 && use_up_wta() && g.D <= 256;
        const int sets = group > 0 ? 2 * l.group : 1;
        for (int i = 0; i < sets; i++) l.vols[i] = take(l.vol_bytes * 8);
        for (int i = 0; i < (l.up_wta ? 3 * l.group : sets); i++) {
            l.cL[i] = take_codes(WH);
            l.cR[i] = take_codes(WH);
        }
        if (l.up_wta)
            for (int i = 0; i < l.group; i++) l.res[i] = take((WH + 64) * 8);
        if (g.width1 > 0) {
            l.n_items[0] = sgm::census_path_items(g, 0xFFu, 1, 1, nullptr, 0);
            l.items[0] = take((size_t)l.n_items[0] * 4);
            if (group > 0) {
                l.n_items[1] = sgm::census_path_items(g, 0xFFu, 1, l.group, nullptr, 0, l.up_wta ? l.group : 0);
                l.items[1] = take((size_t)l.n_items[1] * 4);
            }
        }
    } else {
        // the packed BT planes (16 B/px) only for frames whose cost stage takes the fused kernel
        l.planes = take(sgm::ocv_cost_takes_fused(g) ? sgm::ocv_planes_total(g.W, g.H) : sgm::ocv_planes_bytes(g.W, g.H));
        l.bufA = take(cells * 2);
        l.bufB = take(cells * 2);
        const size_t es = g.wide && !(g.compat & SGM_OCV_SIMD_SAT) ? 4 : 2;   // int32 / int16 path volumes
        // + slack: the path kernel's trash slots (64 lanes x 32 values) and the WTA's last pixel
        // group of the last row, which reads 3 pixels past the volume
        l.ovols = take(es * (sgm::ocv_vol_elems(cells, es) * (p.mode == SGM_MODE_OCV_HH8 ? 8 : 5) + 64 * 32 +
                             (size_t)8 * g.D));
        l.ovf = take(sizeof(int));
        l.ores = take(WH * 8);
    }
    l.tmp = take(WH * 2 * (size_t)std::max(group, 1));   // raw disparity before the median (per frame of a group)
    if (p.speckle_window_size > 0) { l.lab = take(WH * 4); l.cnt = take(WH * 4); }
    if (host_io) { l.inL = take(WH); l.inR = take(WH); l.out = take(WH * 2); l.outf = take(WH * 4); }
    l.total = off;
    return l;
}

// Stage bookkeeping of one match call: begin() before every launch, end() after the last.
struct StageRec {
    sgm_handle* h;
    long open = -1;      // index into h->launches of the launch waiting for its end event
    void close(long ev)
    {
        if (open >= 0 && ev >= 0) h->launches[open].ev1 = (size_t)ev;
        open = -1;
    }
    void begin(const char* name, double bytes)
    {
        const int st = stage_index(h, name, bytes);
        if (!h->profiling) return;
        const long ev = record_event(h);
        close(ev);
        if (st < 0 || ev < 0) return;
        h->launches.push_back({st, (size_t)ev, (size_t)ev});
        open = (long)h->launches.size() - 1;
    }
    void end()
    {
        if (h->profiling && open >= 0) close(record_event(h));
    }
};

// Device work list of the census path launch for (g, only_dir), uploaded on `st` when the
// geometry or the workspace changed. Returns the entry count (< 0: error).
int path_items(sgm_handle* h, const Layout& l, const Geom& g, unsigned dir_mask, int group, hipStream_t st,
               const uint32_t** dev, int up_group = 0)
{
    const int w = group > 1 || up_group > 0 ? 1 : 0;
    uint32_t* d = (uint32_t*)((char*)h->ws.base + l.items[w]);
    *dev = d;
    char key[160];
    snprintf(key, sizeof key, "%d %d %d %d %x %d %d %d %p", g.W, g.H, g.D, g.minD, dir_mask, group, up_group, h->n_cu,
             (void*)d);
    const int n = sgm::census_path_items(g, dir_mask, h->n_cu, group, nullptr, 0, up_group);
    if (h->items_key[w] == key) return n;
    if (n > l.n_items[w]) return fail(h, SGM_ERR_ARG, "path work list larger than its workspace slot");
    if (n > h->items_cap) {
        if (h->items_pin) (void)hipHostFree(h->items_pin);
        h->items_pin = nullptr;
        h->items_cap = 0;
        HIP_TRY(hipHostMalloc((void**)&h->items_pin, (size_t)n * 4, hipHostMallocDefault), "hipHostMalloc");
        h->items_cap = n;
    }
    sgm::census_path_items(g, dir_mask, h->n_cu, group, h->items_pin, h->items_cap, up_group);
    HIP_TRY(hipMemcpyAsync(d, h->items_pin, (size_t)n * 4, hipMemcpyHostToDevice, st), "H2D items");
    HIP_TRY(hipStreamSynchronize(st), "sync");    // geometry changes are rare: never leave the pinned copy in flight
    h->items_key[w] = key;
    return n;
}

// Post filters of one finished frame (src = the WTA output in `tmp` when a median runs).
// tmp_off: element offset of this frame's raw image in `tmp` (a pipelined group holds one
// raw image per frame).
int run_post(sgm_handle* h, const Layout& l, const Geom& g, int16_t* dOut, size_t out_stride, StageRec& rec,
             size_t tmp_off = 0)
{
    const sgm_params& p = h->params;
    char* ws = (char*)h->ws.base;
    const double WH = (double)g.W * g.H;
    const int16_t* raw = (const int16_t*)(ws + l.tmp) + tmp_off;
    const bool med = use_median(p), spk = p.speckle_window_size > 0;
    if (med && !spk) {
        rec.begin("median3", 4 * WH);
        HIP_TRY(sgm::launch_median3(raw, g.W, dOut, out_stride, g.W, g.H, h->stream), "median3");
    }
    if (spk) {   // with a median, the speckle tiles apply it first (one launch less)
        rec.begin(med ? "median3+speckle" : "speckle", (med ? 4 : 0) * WH + 14 * WH);
        HIP_TRY(sgm::launch_speckle(med ? raw : nullptr, g.W, dOut, out_stride, g.W, g.H, g.invalid,
                                    p.speckle_window_size, 16 * p.speckle_range, (int*)(ws + l.lab),
                                    (int*)(ws + l.cnt), h->stream),
                "speckle");
    }
    return SGM_OK;
}

// OpenCV modes: the vertical direction of the last group fused with the WTA (k_ocv_vwta)
// instead of paths + k_ocv_wta16. One wave per column walks H steps and does the pixel WTAs
// itself, so it needs frames with many cells per column chain (interleaved A/B,
// profiles/r03_ocv_vwta_ab.jsonl, ms per frame off -> on: shipped 2448x2048 D=480 MODE_SGBM
// 14.54 -> 13.93, MODE_HH 21.82 -> 21.63; 1080p D=128 MODE_SGBM 1.85 -> 2.11, MODE_HH 2.55 ->
// 2.48; C1 0.23 -> 0.41). SGM_OCV_VWTA = 0 / 1 forces it off / on (parity tests run both).
// D <= 128 with uniqueness < 100 keeps the row WTA in both modes since it is packed
// (k_ocv_wta16_pk, which also lets the paths write deficit volumes): 1080p D=128 MODE_HH
// 2.25 -> 1.97 ms (profiles/r05_ocv_hh_vwta_ab.jsonl), 4096x3000 D=128 MODE_SGBM 9.49-9.65 ->
// 8.63; at 4096x3000 D=256 MODE_HH the fused kernel stays ahead (28.3-28.6 against 30.0 ms,
// profiles/r05_ocv_12mp_vwta_ab.jsonl), so wider ranges keep the thresholds below.
bool ocv_vwta_on(const Geom& g, int fullDP)
{
    if (const char* e = std::getenv("SGM_OCV_VWTA")) return std::atoi(e) != 0;
    if (g.D <= 128 && g.uniq < 100) return false;
    return (double)g.width1 * g.H * g.D >= (fullDP ? 2.0e8 : 1.0e9);
}

// Runs the whole pipeline on device buffers, asynchronously on h->stream.
// copy_r (census mode): dR is not written yet; the left image's census is launched first, then
// copy_r() issues the right image's copy and returns the event that completes it, and the right
// image's census waits on that event (a pageable copy can hold the host until it is done, so the
// left census must already be queued). outf (census mode without median / speckles): the WTA
// writes the final rows as float to outf (a mapped host buffer, row stride outf_stride floats)
// and dOut is not written.
int run_pipeline(sgm_handle* h, const Layout& l, const Geom& g, const uint8_t* dL, const uint8_t* dR, size_t stride,
                 int16_t* dOut, size_t out_stride, const std::function<hipEvent_t()>& copy_r = nullptr,
                 float* outf = nullptr, size_t outf_stride = 0)
{
    const sgm_params& p = h->params;
    char* ws = (char*)h->ws.base;
    hipStream_t st = h->stream;
    const bool med = use_median(p);
    int16_t* tmp = (int16_t*)(ws + l.tmp);
    // the disparity producer writes to `tmp` when a median follows, else directly to dOut
    int16_t* dst = med ? tmp : dOut;
    const size_t dst_stride = med ? (size_t)g.W : out_stride;
    const double WH = (double)g.W * g.H;
    const double cells = (double)std::max(g.width1, 0) * g.H * g.D;
    StageRec rec{h};
    if (h->profiling) h->prof_frames++;
    if (g.width1 <= 0) {
        rec.begin("fill_invalid", 2 * WH);
        HIP_TRY(sgm::launch_fill16(dst, dst_stride, g.W, g.H, g.invalid, st), "fill");
    } else if (p.mode == SGM_MODE_CENSUS8) {
        uint64_t* cL = (uint64_t*)(ws + l.cL[0]);
        uint64_t* cR = (uint64_t*)(ws + l.cR[0]);
        uint8_t* vols = (uint8_t*)(ws + l.vols[0]);
        rec.begin("census", 2 * WH + 16 * WH);
        if (copy_r) {
            HIP_TRY(sgm::launch_census(dL, nullptr, stride, g.W, g.H, cL, nullptr, st), "census L");
            const hipEvent_t r_ready = copy_r();
            if (!r_ready) return SGM_ERR_DEVICE;
            HIP_TRY(hipStreamWaitEvent(st, r_ready, 0), "hipStreamWaitEvent");
            HIP_TRY(sgm::launch_census(dR, nullptr, stride, g.W, g.H, cR, nullptr, st), "census R");
        } else {
            HIP_TRY(sgm::launch_census(dL, dR, stride, g.W, g.H, cL, cR, st), "census");
        }
        const uint32_t* items;
        const int n_items = path_items(h, l, g, 0xFFu, 1, st, &items);
        if (n_items < 0) return n_items;
        sgm::PathFrames pf{};
        pf.cL[0] = cL; pf.cR[0] = cR; pf.vols[0] = vols; pf.n = 1;
        sgm::WtaFrames wf{};
        wf.vols[0] = vols; wf.out[0] = dst; wf.n = 1;
        if (outf) { wf.outf[0] = outf; wf.outf_stride = outf_stride; }
        rec.begin("paths8", 8 * cells);
        HIP_TRY(sgm::launch_census_paths(pf, l.vol_bytes, g, items, n_items, st), "paths");
        rec.begin("wta_lr", 8 * cells + 2 * WH);
        HIP_TRY(sgm::launch_census_wta(wf, l.vol_bytes, g, dst_stride, st), "wta");
    } else {
        const int fullDP = p.mode == SGM_MODE_OCV_HH8;
        const int mask = fullDP ? 0xFF : 0xCD;   // SGBM5: dirs 0,2,3,6,7
        const int ndir = fullDP ? 8 : 5;
        int16_t* A = (int16_t*)(ws + l.bufA);
        int16_t* B = (int16_t*)(ws + l.bufB);
        void* V = ws + l.ovols;
        const size_t ncells = (size_t)g.width1 * g.H * g.D;
        Geom gg = g;
        if (g.wide == 2) {             // the cost kernel raises the flag, the gated launches read it
            gg.ovf = (int*)(ws + l.ovf);
            HIP_TRY(hipMemsetAsync(gg.ovf, 0, sizeof(int), st), "hipMemsetAsync");
        }
        const double es = g.wide == 1 && !(g.compat & SGM_OCV_SIMD_SAT) ? 4 : 2;   // gated: the int16 case
        const bool vwta = ocv_vwta_on(g, fullDP);
        // the plain kernels' volumes as deficit planes where they fit (the stage byte bases below stay
        // those of int16 volumes)
        gg.evol = sgm::ocv_evol_mode(gg, mask, vwta ? sgm::ocv_vwta_dir(ndir) : -1);
        rec.begin("ocv_cost", 2 * WH + 2 * cells);
        HIP_TRY(sgm::launch_ocv_cost(dL, dR, stride, gg, fullDP, (uint8_t*)(ws + l.planes), A, B, st), "ocv_cost");
        if (vwta) {
            // the vertical direction of the last group fused with the WTA (k_ocv_vwta), then
            // disp2 + LR of each row from the per-pixel results (the census rowfin)
            const int fd = sgm::ocv_vwta_dir(ndir);
            uint64_t* res = (uint64_t*)(ws + l.ores);
            // the unfused stages' byte basis (C' counted once, in the paths stage)
            rec.begin("ocv_paths", 2 * cells + es * cells * (ndir - 1));
            HIP_TRY(sgm::launch_ocv_paths(A, A, V, ncells, gg, mask, st, fd), "ocv_paths");
            rec.begin("ocv_vwta", es * cells * (ndir - 1) + 8 * WH);
            HIP_TRY(sgm::launch_ocv_vwta(A, A, V, ncells, ndir, gg, res, st), "ocv_vwta");
            sgm::WtaFrames wf{};
            wf.res[0] = res; wf.out[0] = dst; wf.n = 1;
            rec.begin("ocv_rowfin", 8 * WH + 2 * WH);
            HIP_TRY(sgm::launch_census_rowfin(wf, g, dst_stride, st), "ocv_rowfin");
        } else {
            rec.begin("ocv_paths", 2 * cells + es * cells * ndir);
            HIP_TRY(sgm::launch_ocv_paths(A, A, V, ncells, gg, mask, st), "ocv_paths");
            rec.begin("ocv_wta_lr", es * cells * ndir + 2 * WH);
            HIP_TRY(sgm::launch_ocv_wta(A, V, ncells, ndir, gg, dst, dst_stride, st), "ocv_wta");
        }
    }
    int rc = run_post(h, l, g, dOut, out_stride, rec);
    if (rc) return rc;
    rec.end();
    return SGM_OK;
}

// Callbacks of a frame batch whose inputs arrive and outputs leave while it runs (the
// host-buffer streaming of sgm_match_batch). Frames [f0, f0 + n):
//   inputs       before the first launch that reads their input images;
//   outputs_free before the first launch that writes their disparities;
//   outputs_done after the last launch that writes them.
// Each returns a status (non-zero aborts the batch).
struct FrameHooks {
    virtual int inputs(int f0, int n) = 0;
    virtual int outputs_free(int f0, int n) = 0;
    virtual int outputs_done(int f0, int n) = 0;
    virtual ~FrameHooks() = default;
};

// Frames per pipelined launch: 2 (more path blocks than resident workgroup slots, so the
// dispatcher balances the CUs) unless the batch is shorter; SGM_GROUP overrides (1..4).
int batch_group(int n)
{
    const char* env = std::getenv("SGM_GROUP");
    const int g = env ? std::atoi(env) : 2;
    return std::max(1, std::min({g, sgm::kMaxGroup, n}));
}

// Census-mode frame pipeline on h->stream, in groups of l.group frames.
// up+WTA scheme (l.up_wta, the default):
//   census(G0) | fused[paths7(G0) + census(G1)] | fused[paths7(Gk) + upWTA(Gk-1) + census(Gk+1)]
//   rowfin(Gk-1) post(Gk-1) ... | fused[paths8(Glast) + upWTA(Glast-1)] rowfin post | wta(Glast) post
// paths7 = the seven directions other than dir 1 (volumes written); upWTA = the dir-1 sweep
// of the previous group with its WTA fused (census_sgm.hip UpWta: volume 1 is never stored),
// rowfin = disp2 + LR of those rows. Codes rotate over three sets (group k+1's census runs
// beside group k-1's dir-1 sweep), volumes over two.
// Earlier scheme (SGM_UPWTA=0):
//   census(G0) | fused[paths(G0) + census(G1)] | fused[paths(Gk) + wta(Gk-1) + census(Gk+1)] post(Gk-1)
//   ... | wta(Glast) post
// The census of group k+1 writes the code set of group k-1, whose path sweeps finished in
// the previous launch.
// With a median the WTA of a group writes each frame's raw disparity to its own scratch image
// (post filters read it), so no frame's output is overwritten before its median.
// With h->rect_on, dLs / dRs are raw images (stride = raw stride) rectified inside the census
// (the census tiles read remap(raw)), and rectLs / rectRs (may be null) receive the
// rectified images.
int run_batch_census(sgm_handle* h, const Layout& l, const Geom& g, const uint8_t* const* dLs,
                     const uint8_t* const* dRs, int n, size_t stride, int16_t* const* outs, size_t out_stride,
                     uint8_t* const* rectLs = nullptr, uint8_t* const* rectRs = nullptr, size_t rect_stride = 0,
                     FrameHooks* hooks = nullptr)
{
    const sgm_params& p = h->params;
    char* ws = (char*)h->ws.base;
    hipStream_t st = h->stream;
    const bool med = use_median(p);
    const double WH = (double)g.W * g.H;
    const double cells = (double)g.width1 * g.H * g.D;
    const int G = l.group;
    const bool up = l.up_wta;
    const int ng = (n + G - 1) / G;
    const uint32_t* items;
    const int n_items = path_items(h, l, g, 0xFFu, G, st, &items, up ? G : 0);
    if (n_items < 0) return n_items;
    StageRec rec{h};
    if (h->profiling) h->prof_frames += n;
    auto frames_of = [&](int k) { return std::min(G, n - k * G); };
    auto code_set = [&](int k, int f) { return (up ? k % 3 : k & 1) * G + f; };
    auto path_frames = [&](int k) {
        sgm::PathFrames pf{};
        pf.n = frames_of(k);
        for (int f = 0; f < pf.n; f++) {
            pf.cL[f] = (const uint64_t*)(ws + l.cL[code_set(k, f)]);
            pf.cR[f] = (const uint64_t*)(ws + l.cR[code_set(k, f)]);
            pf.vols[f] = (uint8_t*)(ws + l.vols[(k & 1) * G + f]);
        }
        return pf;
    };
    size_t dst_stride = med ? (size_t)g.W : out_stride;
    auto wta_frames = [&](int k) {
        sgm::WtaFrames wf{};
        wf.n = frames_of(k);
        for (int f = 0; f < wf.n; f++) {
            wf.vols[f] = (const uint8_t*)(ws + l.vols[(k & 1) * G + f]);
            wf.out[f] = med ? (int16_t*)(ws + l.tmp) + (size_t)f * g.W * g.H : outs[k * G + f];
            if (up) {
                wf.cL[f] = (const uint64_t*)(ws + l.cL[code_set(k, f)]);
                wf.cR[f] = (const uint64_t*)(ws + l.cR[code_set(k, f)]);
                wf.res[f] = (uint64_t*)(ws + l.res[f]);
            }
        }
        return wf;
    };
    auto census_frames = [&](int k) {
        sgm::CensusFrames cf{};
        cf.n = frames_of(k);
        cf.stride = stride;
        cf.rect_stride = rect_stride;
        if (h->rect_on) cf.rect = h->rect;
        for (int f = 0; f < cf.n; f++) {
            cf.L[f] = dLs[k * G + f];
            cf.R[f] = dRs[k * G + f];
            cf.cL[f] = (uint64_t*)(ws + l.cL[code_set(k, f)]);
            cf.cR[f] = (uint64_t*)(ws + l.cR[code_set(k, f)]);
            cf.rectL[f] = rectLs ? rectLs[k * G + f] : nullptr;
            cf.rectR[f] = rectRs ? rectRs[k * G + f] : nullptr;
        }
        return cf;
    };
    // hooks of group k (no-ops without hooks)
    auto hk_in = [&](int k) { return hooks ? hooks->inputs(k * G, frames_of(k)) : 0; };
    auto hk_free = [&](int k) { return hooks ? hooks->outputs_free(k * G, frames_of(k)) : 0; };
    auto hk_done = [&](int k) { return hooks ? hooks->outputs_done(k * G, frames_of(k)) : 0; };
    int hrc = hk_in(0);
    if (hrc) return hrc;
    if (h->rect_on) {           // remap + census of the first group, one launch
        rec.begin("rectify+census", (2 * WH + 16 * WH + 16 * WH) * frames_of(0));
        HIP_TRY(sgm::launch_census_tiles(census_frames(0), g.W, g.H, st), "rectify+census");
    } else {
        for (int f = 0; f < frames_of(0); f++) {
            rec.begin("census", 2 * WH + 16 * WH);
            HIP_TRY(sgm::launch_census(dLs[f], dRs[f], stride, g.W, g.H, (uint64_t*)(ws + l.cL[code_set(0, f)]),
                                       (uint64_t*)(ws + l.cR[code_set(0, f)]), st), "census");
        }
    }
    for (int k = 0; k <= ng; k++) {
        // this launch reads the inputs of group k + 1 (census in the tail) and writes the
        // disparities of group k - 1 (WTA, or up+WTA and the row finish after it)
        if (k + 1 < ng && ng > 1 && (hrc = hk_in(k + 1))) return hrc;
        if (k > 0 && (hrc = hk_free(k - 1))) return hrc;
        if (up && k < ng) {
            // the last group sweeps all eight directions (its WTA rows follow alone: a lone
            // launch of up+WTA blocks would be one long latency-bound chain per column block)
            const bool last = k == ng - 1;
            sgm::PathFrames pf = path_frames(k);
            pf.skip_dirs = last ? 0u : 2u;
            const sgm::WtaFrames wf = k > 0 ? wta_frames(k - 1) : sgm::WtaFrames{};
            const sgm::CensusFrames cf = k + 1 < ng ? census_frames(k + 1) : sgm::CensusFrames{};
            // stage name and algorithmic bytes (the canonical dataflow: the dir-1 volume of an
            // up+WTA frame counted as written and read, as if it existed) from the launch's parts
            const char* name = last ? (wf.n ? "paths8+up_wta" : "paths8")
                                    : (wf.n ? (cf.n ? "paths7+up_wta+census" : "paths7+up_wta")
                                            : (cf.n ? "paths7+census" : "paths7"));
            rec.begin(name, (last ? 8 : 7) * cells * pf.n + (9 * cells + 2 * WH) * wf.n + 18 * WH * cf.n);
            HIP_TRY(sgm::launch_census_fused(pf, wf, cf, l.vol_bytes, g, items, n_items, dst_stride, true, st),
                    "fused");
            if (wf.n) {
                rec.begin("rowfin", 10 * WH * wf.n);
                HIP_TRY(sgm::launch_census_rowfin(wf, g, dst_stride, st), "rowfin");
            }
        } else if (k == ng) {
            rec.begin("wta_lr", (8 * cells + 2 * WH) * frames_of(k - 1));
            HIP_TRY(sgm::launch_census_wta(wta_frames(k - 1), l.vol_bytes, g, dst_stride, st), "wta");
        } else if (ng == 1) {
            rec.begin("paths8", 8 * cells * frames_of(0));
            HIP_TRY(sgm::launch_census_paths(path_frames(0), l.vol_bytes, g, items, n_items, st), "paths");
        } else {
            const sgm::WtaFrames wf = k > 0 ? wta_frames(k - 1) : sgm::WtaFrames{};
            const sgm::CensusFrames cf = k + 1 < ng ? census_frames(k + 1) : sgm::CensusFrames{};
            const char* name = wf.n ? (cf.n ? "paths8+wta_lr+census" : "paths8+wta_lr") : "paths8+census";
            rec.begin(name, 8 * cells * frames_of(k) + (8 * cells + 2 * WH) * wf.n + 18 * WH * cf.n);
            HIP_TRY(sgm::launch_census_fused(path_frames(k), wf, cf, l.vol_bytes, g, items, n_items, dst_stride, false,
                                             st),
                    "fused");
        }
        if (k > 0) {
            const int k1 = k - 1;
            for (int f = 0; f < frames_of(k1); f++) {
                int rc = run_post(h, l, g, outs[k1 * G + f], out_stride, rec, (size_t)f * g.W * g.H);
                if (rc) return rc;
            }
            if ((hrc = hk_done(k1))) return hrc;
        }
    }
    rec.end();
    return SGM_OK;
}

int prepare(sgm_handle* h, int W, int H, bool host_io, Geom& g, Layout& l, int group = 0)
{
    int rc = make_geom(h->params, W, H, g, h->err);
    if (rc) return rc;
    if ((rc = ensure_stream(h))) return rc;
    l = make_layout(h->params, g, host_io, group);
    // the uploaded path work list lives in the workspace: any other use of it invalidates it
    if (h->params.mode != SGM_MODE_CENSUS8) { h->items_key[0].clear(); h->items_key[1].clear(); }
    return ensure_ws(h, l.total);
}

// OCV-mode batch (sgm_match_device_batch on an OpenCV mode): frames dealt round-robin over
// S same-device lanes (own stream + workspace each; SGM_OCV_STREAMS, default 4, 1 = one
// frame after another on the handle's stream). Lane 0 is h itself (its workspace is the one
// the caller prepared); lanes 1.. are sub-handles, opened only while the device's free memory
// holds their workspace (the shipped 2448x2048 D=480 block-21 frame needs 27-70 GB per
// workspace, by mode and OpenCV build), and a lane whose allocation fails ends the list. Every
// lane starts after the work already on h->stream, and h->stream waits for every lane, so the
// call keeps the single-stream contract.
int ocv_batch_lanes(int n)
{
    const char* e = std::getenv("SGM_OCV_STREAMS");
    const int s = e ? std::atoi(e) : 4;
    return std::max(1, std::min({s, n, 8}));
}

int run_batch_ocv(sgm_handle* h, const Layout& l0, const Geom& g0, int W, int H, const uint8_t* const* dLs,
                  const uint8_t* const* dRs, int n, size_t stride, int16_t* const* outs, size_t out_stride)
{
    const int Smax = ocv_batch_lanes(n);
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    const size_t reserve = std::max<size_t>(total_b / 64, (size_t)1 << 30);   // headroom for the caller
    std::vector<Geom> g(1, g0);
    std::vector<Layout> l(1, l0);
    while ((int)h->par.size() < Smax - 1) h->par.push_back(nullptr);
    int S = 1;
    for (int s = 1; s < Smax; s++) {
        sgm_handle*& q = h->par[s - 1];
        const size_t have = q ? q->ws.size : 0;
        const size_t extra = have >= l0.total ? 0 : l0.total;
        if (extra + reserve > free_b) break;
        if (!q && sgm_create(&q, h->device) != SGM_OK) break;
        q->params = h->params;
        Geom gq;
        Layout lq;
        if (prepare(q, W, H, false, gq, lq) != SGM_OK) {   // e.g. an allocation failure: fewer lanes
            q->err.clear();
            break;
        }
        free_b -= std::min(free_b, extra);
        g.push_back(gq);
        l.push_back(lq);
        S = s + 1;
    }
    if (S > 1) {
        if (!h->par_ev) HIP_TRY(hipEventCreateWithFlags(&h->par_ev, hipEventDisableTiming), "hipEventCreate");
        HIP_TRY(hipEventRecord(h->par_ev, h->stream), "hipEventRecord");
        for (int s = 1; s < S; s++) HIP_TRY(hipStreamWaitEvent(h->par[s - 1]->stream, h->par_ev, 0), "hipStreamWaitEvent");
    }
    for (int i = 0; i < n; i++) {
        const int s = i % S;
        sgm_handle* q = s ? h->par[s - 1] : h;
        const int rc = run_pipeline(q, l[s], g[s], dLs[i], dRs[i], stride, outs[i], out_stride);
        if (rc) return q == h ? rc : fail(h, rc, q->err);
    }
    for (int s = 1; s < S; s++) {
        sgm_handle* q = h->par[s - 1];
        HIP_TRY(hipEventRecord(q->done, q->stream), "hipEventRecord");
        q->done_stream = q->stream;
        HIP_TRY(hipStreamWaitEvent(h->stream, q->done, 0), "hipStreamWaitEvent");
    }
    // lanes whose workspaces take more than a quarter of the device are not kept past the call
    // (a later call on h, or another handle, may need that memory): the call waits for them
    // (SGM_OCV_KEEP_LANES=1 keeps them: the A/B of profiles/r04_ocv_lanes_ab.jsonl)
    const char* keep = std::getenv("SGM_OCV_KEEP_LANES");
    if ((size_t)(S - 1) * l0.total > total_b / 4 && !(keep && std::atoi(keep))) {
        for (int s = 1; s < S; s++) {
            sgm_handle* q = h->par[s - 1];
            HIP_TRY(hipStreamSynchronize(q->stream), "hipStreamSynchronize");
            HIP_TRY(hipFree(q->ws.base), "hipFree lane workspace");
            q->ws = Workspace{};
            q->items_key[0].clear();
            q->items_key[1].clear();
        }
    }
    return SGM_OK;
}

// Host images in, host disparity out (sgm_match: int16; sgm_match_f32: the CV_32FC1 the
// node's matcher contract wants, converted on the device). The reference's path is
// matcherOpenCVSGBM.cpp:17-44 (compute, then convertTo CV_32FC1), called per frame from
// generate_disparity.cpp:334-368. Every copy is one 2-D DMA between the caller's (pageable)
// rows and the workspace: measured on the MI355X box (tools/probe/host_copy.cpp,
// profiles/r04_host_copy.txt), a pageable 1920x1080 H2D takes 58 us against 42 us of CPU
// packing + 45 us of pinned DMA, and the 8.3 MB float D2H runs at the same 53 GB/s into
// pageable or pinned memory — staging buffers would only add copies.
// A caller may page-lock `out` with sgm_host_register (the adapter does, for its persistent
// disparity_lr): the D2H then needs no runtime staging, 1920x1080 f32 forwardMatch 1.95-1.97
// vs 1.97-1.99 ms pageable (profiles/r04_host_copy_ab.jsonl). Copying the rows back in 4 bands
// behind a banded WTA measured no gain (1.97-2.00 ms): a quarter-frame WTA launch (270 row
// workgroups) runs below the full launch's efficiency by about what the overlap saves.
int match_host(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, void* out,
               size_t out_stride, bool f32)
{
    Geom g;
    Layout l;
    int rc = prepare(h, W, H, true, g, l);
    if (rc || (rc = order_after_last(h, h->stream))) return rc;
    hipStream_t st = h->stream;
    const size_t es = f32 ? 4 : 2;
    char* ws = (char*)h->ws.base;
    const sgm_params& p = h->params;
    const bool census = p.mode == SGM_MODE_CENSUS8 && g.width1 > 0;
    // census mode: the left image's census runs while the right image is copied (second stream)
    if (census) {
        if (!h->cpy) HIP_TRY(hipStreamCreateWithFlags(&h->cpy, hipStreamNonBlocking), "hipStreamCreate");
        if (!h->cpy_ev) HIP_TRY(hipEventCreateWithFlags(&h->cpy_ev, hipEventDisableTiming), "hipEventCreate");
        HIP_TRY(hipEventRecord(h->cpy_ev, st), "hipEventRecord");        // the workspace is free
        HIP_TRY(hipStreamWaitEvent(h->cpy, h->cpy_ev, 0), "hipStreamWaitEvent");
    }
    HIP_TRY(hipMemcpy2DAsync(ws + l.inL, W, L, stride, W, H, hipMemcpyHostToDevice, st), "H2D L");
    // f32 output that is the WTA's own (census, no median / speckles) into a registered, mapped
    // host buffer: the WTA writes the float rows there itself (no to-float pass, no copy back)
    float* outf = nullptr;
    if (f32 && census && !use_median(p) && p.speckle_window_size <= 0) {
        const size_t need = out_stride * 4 * (size_t)(H - 1) + (size_t)W * 4;
        for (const auto& r : h->regs)
            if (r.dev && (char*)out >= r.host && (char*)out + need <= r.host + r.bytes) {
                outf = (float*)(r.dev + ((char*)out - r.host));
                break;
            }
    }
    int16_t* d16 = (int16_t*)(ws + l.out);
    std::function<hipEvent_t()> copy_r;
    if (census) {
        copy_r = [&]() -> hipEvent_t {
            hipError_t e = hipMemcpy2DAsync(ws + l.inR, W, R, stride, W, H, hipMemcpyHostToDevice, h->cpy);
            if (e == hipSuccess) e = hipEventRecord(h->cpy_ev, h->cpy);
            if (e != hipSuccess) { hip_fail(h, e, "H2D R"); return nullptr; }
            return h->cpy_ev;
        };
    } else {
        HIP_TRY(hipMemcpy2DAsync(ws + l.inR, W, R, stride, W, H, hipMemcpyHostToDevice, st), "H2D R");
    }
    rc = run_pipeline(h, l, g, (const uint8_t*)(ws + l.inL), (const uint8_t*)(ws + l.inR), W, d16, W, copy_r, outf,
                      out_stride);
    if (rc) return rc;
    if (outf) {
        HIP_TRY(hipStreamSynchronize(st), "sync");
        return mark_done(h, st);
    }
    const void* dsrc = d16;
    if (f32) {
        HIP_TRY(sgm::launch_to_f32(d16, W, (float*)(ws + l.outf), W, W, H, st), "to_f32");
        dsrc = ws + l.outf;
    }
    HIP_TRY(hipMemcpy2DAsync(out, out_stride * es, dsrc, W * es, W * es, H, hipMemcpyDeviceToHost, st), "D2H");
    HIP_TRY(hipStreamSynchronize(st), "sync");
    return mark_done(h, st);
}

}  // namespace

// ==================================================================================== C-ABI
extern "C" {

int sgm_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void sgm_default_params(sgm_params* p, int mode)
{
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->mode = mode;
    if (mode == SGM_MODE_CENSUS8) {
        p->min_disparity = 0; p->num_disparities = 128; p->p1 = 10; p->p2 = 120;
        p->uniqueness_ratio = 5; p->disp12_max_diff = 1; p->subpixel = 1; p->lr_check = 1; p->median = 0;
    } else {
        // generate_disparity.cpp:100-112 node defaults
        p->min_disparity = 9; p->num_disparities = 64; p->block_size = 15; p->p1 = 200; p->p2 = 400;
        p->uniqueness_ratio = 15; p->disp12_max_diff = 0; p->prefilter_cap = 31; p->speckle_window_size = 100;
        p->speckle_range = 4; p->subpixel = 1; p->lr_check = 1; p->median = 1;
        p->ocv_compat = SGM_OCV_COMPAT_MELODIC;   // the reference's Dockerfile:1 (melodic, OpenCV 3.2 SSE2)
    }
}

int sgm_create(sgm_handle** out, int device)
{
    if (!out) return SGM_ERR_ARG;
    *out = nullptr;
    const int n = sgm_device_count();
    if (device < 0 || device >= n) return SGM_ERR_DEVICE;
    sgm_handle* h = new (std::nothrow) sgm_handle();
    if (!h) return SGM_ERR_ALLOC;
    h->device = device;
    sgm_default_params(&h->params, SGM_MODE_CENSUS8);
    *out = h;
    return SGM_OK;
}

void sgm_destroy(sgm_handle* h)
{
    if (!h) return;
    for (sgm_handle* s : h->sub) sgm_destroy(s);
    for (sgm_handle* s : h->bands) sgm_destroy(s);
    for (sgm_handle* s : h->par) sgm_destroy(s);
    if (hipSetDevice(h->device) == hipSuccess) {
        if (h->par_ev) (void)hipEventDestroy(h->par_ev);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        if (h->stream2) (void)hipStreamSynchronize(h->stream2);
        if (h->done_stream) (void)hipEventSynchronize(h->done);   // the last call on a caller's stream
        for (hipEvent_t e : h->bev) if (e) (void)hipEventDestroy(e);
        if (h->stream2) (void)hipStreamDestroy(h->stream2);
        if (h->ws.base) (void)hipFree(h->ws.base);
        if (h->pin) (void)hipHostFree(h->pin);
        if (h->items_pin) (void)hipHostFree(h->items_pin);
        if (h->aux) (void)hipFree(h->aux);
        if (h->cubic_tab) (void)hipFree(h->cubic_tab);
        for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
        if (h->up) { (void)hipStreamSynchronize(h->up); (void)hipStreamDestroy(h->up); }
        if (h->down) { (void)hipStreamSynchronize(h->down); (void)hipStreamDestroy(h->down); }
        for (hipEvent_t e : h->io_ev) (void)hipEventDestroy(e);
        if (h->io_dev) (void)hipFree(h->io_dev);
        if (h->io_pin) (void)hipHostFree(h->io_pin);
        if (h->cpy) { (void)hipStreamSynchronize(h->cpy); (void)hipStreamDestroy(h->cpy); }
        if (h->cpy_ev) (void)hipEventDestroy(h->cpy_ev);
        for (const auto& r : h->regs) (void)hipHostUnregister(r.host);
        if (h->done) (void)hipEventDestroy(h->done);
        if (h->stream) (void)hipStreamDestroy(h->stream);
    }
    delete h;
}

int sgm_set_params(sgm_handle* h, const sgm_params* p)
{
    if (!h || !p) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    h->params = *p;
    return SGM_OK;
}

int sgm_get_params(const sgm_handle* h, sgm_params* p)
{
    if (!h || !p) return SGM_ERR_ARG;
    *p = h->params;
    return SGM_OK;
}

int sgm_abi_version(void) { return SGM_ABI_VERSION; }

int sgm_host_register(sgm_handle* h, void* ptr, size_t bytes)
{
    if (!h) return SGM_ERR_ARG;
    if (!ptr || !bytes) return fail(h, SGM_ERR_ARG, "null or empty host range");
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    // a failed registration is not fatal to the caller (it falls back to pageable copies), so
    // HIP's last error is cleared here: the next launcher's hipGetLastError must not report it
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return hip_fail(h, e, "hipHostRegister");
    }
    void* dev = nullptr;
    if ((e = hipHostGetDevicePointer(&dev, ptr, 0)) != hipSuccess) dev = nullptr;   // registered, not mapped
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lk(h->mu);
    h->regs.push_back({(char*)ptr, bytes, (char*)dev});
    return SGM_OK;
}

int sgm_host_unregister(sgm_handle* h, void* ptr)
{
    if (!h) return SGM_ERR_ARG;
    if (!ptr) return fail(h, SGM_ERR_ARG, "null host pointer");
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->done_stream) HIP_TRY(hipEventSynchronize(h->done), "hipEventSynchronize");   // no kernel still writes it
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) {                 // still registered: the handle keeps its mapping
        (void)hipGetLastError();
        return hip_fail(h, e, "hipHostUnregister");
    }
    for (size_t i = 0; i < h->regs.size(); i++)
        if (h->regs[i].host == (char*)ptr) { h->regs.erase(h->regs.begin() + i); break; }
    return SGM_OK;
}

int sgm_check_params(const sgm_params* p, int width, int height)
{
    if (!p) return SGM_ERR_ARG;
    Geom g;
    std::string err;
    return make_geom(*p, width, height, g, err);
}

const char* sgm_last_error(const sgm_handle* h) { return h ? h->err.c_str() : "null handle"; }

int sgm_match_device(sgm_handle* h, const uint8_t* dL, const uint8_t* dR, int W, int H, size_t stride, int16_t* dOut,
                     size_t out_stride, void* stream)
{
    if (!h) return SGM_ERR_ARG;
    if (h->rect_on) {          // raw inputs: the census-fused rectification path
        const uint8_t* l1[1] = {dL};
        const uint8_t* r1[1] = {dR};
        int16_t* o1[1] = {dOut};
        return sgm_match_device_batch_rect(h, l1, r1, 1, W, H, stride, nullptr, nullptr, 0, o1, out_stride, stream);
    }
    std::lock_guard<std::mutex> lk(h->mu);
    if (!dL || !dR || !dOut || stride < (size_t)W || out_stride < (size_t)W) return fail(h, SGM_ERR_ARG, "bad buffers");
    Geom g;
    Layout l;
    int rc = prepare(h, W, H, false, g, l);
    if (rc) return rc;
    hipStream_t own = h->stream;
    if (stream) h->stream = (hipStream_t)stream;
    rc = order_after_last(h, h->stream);
    if (!rc) rc = run_pipeline(h, l, g, dL, dR, stride, dOut, out_stride);
    if (!rc) rc = mark_done(h, h->stream);
    h->stream = own;
    return rc;
}

int sgm_match_device_batch_rect(sgm_handle* h, const uint8_t* const* dLs, const uint8_t* const* dRs, int n, int W,
                                int H, size_t stride, uint8_t* const* rectLs, uint8_t* const* rectRs,
                                size_t rect_stride, int16_t* const* outs, size_t out_stride, void* stream)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    const size_t in_w = h->rect_on ? (size_t)h->rect.src_w : (size_t)W;
    if (n < 0 || (n > 0 && (!dLs || !dRs || !outs)) || stride < in_w || out_stride < (size_t)W)
        return fail(h, SGM_ERR_ARG, "bad buffers");
    if ((rectLs || rectRs) && (!h->rect_on || rect_stride < (size_t)W))
        return fail(h, SGM_ERR_ARG, "rectified outputs need sgm_set_rectification and rect_stride >= width");
    for (int i = 0; i < n; i++)
        if (!dLs[i] || !dRs[i] || !outs[i]) return fail(h, SGM_ERR_ARG, "null frame pointer");
    if (n == 0) return SGM_OK;
    if (h->rect_on && h->params.mode != SGM_MODE_CENSUS8)
        return fail(h, SGM_ERR_UNSUPPORTED, "fused rectification runs in the census mode (use sgm_remap_cubic)");
    Geom g;
    Layout l;
    int rc = make_geom(h->params, W, H, g, h->err);
    if (rc) return rc;
    if (h->rect_on && g.width1 <= 0)
        return fail(h, SGM_ERR_UNSUPPORTED, "fused rectification needs a non-empty disparity window");
    const bool pipelined = h->params.mode == SGM_MODE_CENSUS8 && (n >= 2 || h->rect_on) && g.width1 > 0;
    rc = prepare(h, W, H, false, g, l, pipelined ? batch_group(n) : 0);
    if (rc) return rc;
    hipStream_t own = h->stream;
    if (stream) h->stream = (hipStream_t)stream;
    rc = order_after_last(h, h->stream);
    if (rc) {
    } else if (pipelined) {
        rc = run_batch_census(h, l, g, dLs, dRs, n, stride, outs, out_stride, rectLs, rectRs, rect_stride);
    } else if (h->params.mode != SGM_MODE_CENSUS8 && ocv_batch_lanes(n) > 1 && !h->profiling) {
        rc = run_batch_ocv(h, l, g, W, H, dLs, dRs, n, stride, outs, out_stride);
    } else {
        for (int i = 0; i < n && rc == 0; i++) rc = run_pipeline(h, l, g, dLs[i], dRs[i], stride, outs[i], out_stride);
    }
    if (!rc) rc = mark_done(h, h->stream);
    h->stream = own;
    return rc;
}

int sgm_match_device_batch(sgm_handle* h, const uint8_t* const* dLs, const uint8_t* const* dRs, int n, int W, int H,
                           size_t stride, int16_t* const* outs, size_t out_stride, void* stream)
{
    return sgm_match_device_batch_rect(h, dLs, dRs, n, W, H, stride, nullptr, nullptr, 0, outs, out_stride, stream);
}

int sgm_set_rectification(sgm_handle* h, const float* d_map_xl, const float* d_map_yl, const float* d_map_xr,
                          const float* d_map_yr, size_t map_stride, int src_w, int src_h)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!d_map_xl && !d_map_yl && !d_map_xr && !d_map_yr) { h->rect_on = false; return SGM_OK; }
    if (!d_map_xl || !d_map_yl || !d_map_xr || !d_map_yr || src_w <= 0 || src_h <= 0 || map_stride == 0)
        return fail(h, SGM_ERR_ARG, "rectification needs four maps and the raw image size");
    int rc = ensure_stream(h);
    if (rc) return rc;
    if ((rc = ensure_cubic_table(h))) return rc;
    h->rect = sgm::RectifyIn{{d_map_xl, d_map_yl, d_map_xr, d_map_yr}, map_stride, src_w, src_h, h->cubic_tab};
    h->rect_on = true;
    return SGM_OK;
}

int sgm_disparity_to_msg(sgm_handle* h, const int16_t* d_disp, size_t disp_stride, int W, int H, float min_disparity,
                         float max_disparity, float* d_out, size_t out_stride, void* stream)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!d_disp || !d_out || W <= 0 || H <= 0 || disp_stride < (size_t)W || out_stride < (size_t)W)
        return fail(h, SGM_ERR_ARG, "bad buffers or sizes");
    int rc = ensure_stream(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    HIP_TRY(sgm::launch_disp_to_msg(d_disp, disp_stride, W, H, min_disparity, max_disparity, d_out, out_stride, st),
            "disp_to_msg");
    return SGM_OK;
}

int sgm_rectify_map(sgm_handle* h, const double K[9], const double* dist, int n_dist, const double R[9],
                    const double P[12], int W, int H, float* d_map_x, float* d_map_y, size_t map_stride, void* stream)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!K || !P || !d_map_x || !d_map_y || W <= 0 || H <= 0 || map_stride < (size_t)W || (n_dist > 0 && !dist))
        return fail(h, SGM_ERR_ARG, "bad buffers or sizes");
    if (n_dist != 0 && n_dist != 4 && n_dist != 5 && n_dist != 8 && n_dist != 12)
        return fail(h, SGM_ERR_UNSUPPORTED, "distortion vector must have 0, 4, 5, 8 or 12 elements");
    double d12[12] = {};
    for (int i = 0; i < n_dist; i++) d12[i] = dist[i];
    double ir[9];
    if (!sgm::rectify_inverse(P, R, ir)) return fail(h, SGM_ERR_ARG, "singular P[:, :3] * R");
    int rc = ensure_stream(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    HIP_TRY(sgm::launch_rectify_map(K, d12, ir, W, H, d_map_x, d_map_y, map_stride, st), "rectify_map");
    return SGM_OK;
}

void sgm_cubic_table(int16_t* tab) { if (tab) sgm::cubic_table(tab); }

int sgm_remap_cubic(sgm_handle* h, const uint8_t* d_src, size_t src_stride, int src_w, int src_h, const float* d_map_x,
                    const float* d_map_y, size_t map_stride, int W, int H, uint8_t* d_dst, size_t dst_stride,
                    void* stream)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!d_src || !d_map_x || !d_map_y || !d_dst || W <= 0 || H <= 0 || src_w <= 0 || src_h <= 0 ||
        src_stride < (size_t)src_w || map_stride < (size_t)W || dst_stride < (size_t)W)
        return fail(h, SGM_ERR_ARG, "bad buffers or sizes");
    int rc = ensure_stream(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if ((rc = ensure_cubic_table(h))) return rc;
    HIP_TRY(sgm::launch_remap_cubic(d_src, src_stride, src_w, src_h, d_map_x, d_map_y, map_stride, W, H,
                                    h->cubic_tab, d_dst, dst_stride, st), "remap_cubic");
    return SGM_OK;
}

void sgm_calc_q(const double K[9], const double Pr[12], const double Pl[12], double Q[16])
{
    // disparity_to_depth.cpp:62-84
    const double cx = Pl[2], cxr = Pr[2], cy = Pl[4 + 2], fx = K[0];
    const double p14 = Pr[3];
    const double T = -p14 / fx;
    const double q33 = -(cx - cxr) / T;
    for (int i = 0; i < 16; i++) Q[i] = 0.0;
    Q[0] = 1.0;  Q[3] = -cx;
    Q[5] = 1.0;  Q[7] = -cy;
    Q[11] = fx;
    Q[14] = 1.0 / T;
    Q[15] = q33;
}

int sgm_depth_points(sgm_handle* h, const float* d_disp, size_t disp_stride, int W, int H, const uint8_t* d_color,
                     size_t color_stride, int channels, const double q[5], double depth_min, double depth_max,
                     float* d_depth, size_t depth_stride, sgm_point_xyzrgb* d_points, int max_points,
                     int* d_num_points, void* stream)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!d_disp || !q || W <= 0 || H <= 0 || disp_stride < (size_t)W || (d_depth && depth_stride < (size_t)W) ||
        (channels != 0 && channels != 1 && channels != 3) || (channels && !d_color) ||
        (channels && color_stride < (size_t)W * channels) || (d_points && max_points < 0))
        return fail(h, SGM_ERR_ARG, "bad buffers or sizes");
    int rc = ensure_stream(h);
    if (rc) return rc;
    if (h->aux_n < (size_t)(2 * H + 1)) {
        if (h->aux) (void)hipFree(h->aux);
        h->aux = nullptr;
        h->aux_n = 0;
        HIP_TRY(hipMalloc(&h->aux, sizeof(int) * (2 * (size_t)H + 1)), "hipMalloc aux");
        h->aux_n = 2 * (size_t)H + 1;
    }
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    const float qf[5] = {(float)q[0], (float)q[1], (float)q[2], (float)q[3], (float)q[4]};   // :134-138
    int* row_count = h->aux;
    int* row_off = h->aux + H;
    HIP_TRY(sgm::launch_depth_points(d_disp, disp_stride, W, H, qf, depth_min, depth_max, d_color, color_stride,
                                     channels, d_depth, depth_stride, (float4*)d_points, d_points ? max_points : 0,
                                     row_count, row_off, st), "depth_points");
    if (d_num_points)
        HIP_TRY(hipMemcpyAsync(d_num_points, row_off + H, sizeof(int), hipMemcpyDeviceToDevice, st), "count");
    return SGM_OK;
}

int sgm_synchronize(sgm_handle* h)
{
    if (!h) return SGM_ERR_ARG;
    if (!h->stream) return SGM_OK;
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    HIP_TRY(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    return SGM_OK;
}

int sgm_match(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, int16_t* disp,
              size_t out_stride)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->rect_on) return fail(h, SGM_ERR_UNSUPPORTED, "fused rectification applies to device-buffer matches");
    if (!L || !R || !disp || W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W)
        return fail(h, SGM_ERR_ARG, "bad buffers or sizes");
    return match_host(h, L, R, W, H, stride, disp, out_stride, false);
}

int sgm_match_f32(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, float* disp,
                  size_t out_stride)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->rect_on) return fail(h, SGM_ERR_UNSUPPORTED, "fused rectification applies to device-buffer matches");
    if (!L || !R || !disp || W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W)
        return fail(h, SGM_ERR_ARG, "bad buffers or sizes");
    return match_host(h, L, R, W, H, stride, disp, out_stride, true);
}

}  // extern "C"

// Per-device sub-handles (created on demand, parameters copied from h); devs = the devices.
static int open_subs(sgm_handle* h, const int* devices, int n_dev, std::vector<int>& devs)
{
    devs.clear();
    if (!devices || n_dev <= 0) {
        const int n = sgm_device_count();
        for (int i = 0; i < n; i++) devs.push_back(i);
    } else {
        devs.assign(devices, devices + n_dev);
    }
    if (devs.empty()) return fail(h, SGM_ERR_DEVICE, "no HIP device");
    std::lock_guard<std::mutex> lk(h->mu);
    while (h->sub.size() < devs.size()) h->sub.push_back(nullptr);
    for (size_t i = 0; i < devs.size(); i++) {
        if (h->sub[i] && h->sub[i]->device != devs[i]) { sgm_destroy(h->sub[i]); h->sub[i] = nullptr; }
        if (!h->sub[i]) {
            int rc = sgm_create(&h->sub[i], devs[i]);
            if (rc) return fail(h, rc, "cannot open device " + std::to_string(devs[i]));
        }
        h->sub[i]->params = h->params;
    }
    return SGM_OK;
}

// Runs job(t, sub-handle) on one host thread per device; first error wins.
template <typename F>
static int run_on_subs(sgm_handle* h, const std::vector<int>& devs, F job)
{
    std::vector<int> rcs(devs.size(), SGM_OK);
    std::vector<std::thread> th;
    for (size_t t = 0; t < devs.size(); t++) th.emplace_back([&, t]() { rcs[t] = job((int)t, h->sub[t]); });
    for (auto& t : th) t.join();
    for (size_t t = 0; t < devs.size(); t++)
        if (rcs[t]) return fail(h, rcs[t], std::string("device ") + std::to_string(devs[t]) + ": " + h->sub[t]->err);
    return SGM_OK;
}

// ------------------------------------------------------- host-buffer frame streaming ----
// sgm_match_batch on one device (SURVEY §8(e) "frame batch": one host thread + stream set
// per device, pinned host rings). The device's frames flow through rings of pinned host
// slots and device slots (io_ring_frames) while the pipelined batch runs:
//   packer thread    user L/R rows -> pinned input slot (once that slot's previous H2D is done)
//   driver (caller)  H2D on `up` -> census / paths / WTA / post on the compute stream -> D2H on `down`
//   unpacker thread  pinned output slot -> user disparity rows (once its D2H is done)
// so the host copies, both PCIe directions and the kernels overlap; the driver only blocks
// when a ring is full. The copies run as blit kernels on high-priority streams, so they
// slip in between the pipeline launch's workgroups instead of waiting for it to end
// (C3 host-buffer batch: 530 -> 629 pairs/s against 664 device-resident). Reference pattern: the per-frame upload/match/download of
// matcherOpenCVBlockCuda.cpp:27-30, driven per frame by generate_disparity.cpp:334-368.
namespace {

constexpr int kIoRing = 16;   // max frames per ring

// Frames per ring: up to 256 MB of pinned staging per device, at least 8 frames (> 2 groups
// of sgm::kMaxGroup frames, so a launch never waits on its own group's slots).
int io_ring_frames(size_t WH) { return (int)std::max<size_t>(8, std::min<size_t>(kIoRing, (256u << 20) / (4 * WH))); }

struct HostStreamer final : FrameHooks {
    sgm_handle* h = nullptr;
    int W = 0, H = 0;
    size_t stride = 0, out_stride = 0, WH = 0;
    std::vector<const uint8_t*> L, R;   // this device's frames, local order
    std::vector<int16_t*> O;
    int n = 0;
    int ring = kIoRing;              // frames per ring (io_ring_frames)
    uint8_t* din = nullptr;             // device ring: ring x (left | right)
    int16_t* dout = nullptr;            // device ring: ring x disparity
    uint8_t* pin = nullptr;             // pinned ring: ring x (left | right)
    int16_t* pout = nullptr;            // pinned ring: ring x disparity
    hipEvent_t *ev_h2d = nullptr, *ev_free = nullptr, *ev_d2h = nullptr, ev_ready = nullptr;   // per slot
    std::mutex m;
    std::condition_variable cv;
    // progress counters (frames): packed into pinned slots, H2D issued, read by an issued
    // launch, D2H issued, copied to the caller
    int packed = 0, uploaded = 0, consumed = 0, d2h_issued = 0, unpacked = 0;
    int err = SGM_OK;
    std::string err_msg;
    bool stop = false;
    // SGM_IO_TRACE=1: seconds spent copying / waiting per role, printed after the batch
    double t_pack = 0, t_pack_wait = 0, t_unpack = 0, t_unpack_wait = 0, t_drv_in = 0, t_drv_out = 0;
    double t_api_in = 0, t_api_free = 0, t_api_out = 0;   // inside the HIP calls of each hook
    static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

    void set_error(int code, const std::string& msg)
    {
        std::lock_guard<std::mutex> lk(m);
        if (!err) { err = code; err_msg = msg; }
        stop = true;
        cv.notify_all();
    }
    int hip_error(hipError_t e, const char* where)
    {
        set_error(SGM_ERR_DEVICE, std::string(where) + ": " + hipGetErrorString(e));
        return SGM_ERR_DEVICE;
    }
    // blocks until pred() or a stop; false on stop
    template <typename P> bool wait_for(P pred)
    {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop || pred(); });
        return !stop;
    }
    void advance(int& counter, int v)
    {
        { std::lock_guard<std::mutex> lk(m); counter = v; }
        cv.notify_all();
    }

    void packer()
    {
        if (hipSetDevice(h->device) != hipSuccess) { set_error(SGM_ERR_DEVICE, "hipSetDevice"); return; }
        for (int j = 0; j < n; j++) {
            const int slot = j % ring;
            double t0 = now();
            if (j >= ring) {            // the slot's previous frame must have left for the device
                if (!wait_for([&] { return uploaded > j - ring; })) return;
                hipError_t e = hipEventSynchronize(ev_h2d[slot]);
                if (e != hipSuccess) { hip_error(e, "packer: hipEventSynchronize"); return; }
            }
            double t1 = now();
            t_pack_wait += t1 - t0;
            uint8_t* dst = pin + (size_t)slot * 2 * WH;
            if (stride == (size_t)W) {
                std::memcpy(dst, L[j], WH);
                std::memcpy(dst + WH, R[j], WH);
            } else {
                for (int y = 0; y < H; y++) std::memcpy(dst + (size_t)y * W, L[j] + (size_t)y * stride, W);
                for (int y = 0; y < H; y++) std::memcpy(dst + WH + (size_t)y * W, R[j] + (size_t)y * stride, W);
            }
            t_pack += now() - t1;
            advance(packed, j + 1);
        }
    }

    void unpacker()
    {
        if (hipSetDevice(h->device) != hipSuccess) { set_error(SGM_ERR_DEVICE, "hipSetDevice"); return; }
        for (int j = 0; j < n; j++) {
            double t0 = now();
            if (!wait_for([&] { return d2h_issued > j; })) return;
            const int slot = j % ring;
            hipError_t e = hipEventSynchronize(ev_d2h[slot]);
            if (e != hipSuccess) { hip_error(e, "unpacker: hipEventSynchronize"); return; }
            double t1 = now();
            t_unpack_wait += t1 - t0;
            const int16_t* src = pout + (size_t)slot * WH;
            if (out_stride == (size_t)W) {
                std::memcpy(O[j], src, WH * 2);
            } else {
                for (int y = 0; y < H; y++) std::memcpy(O[j] + (size_t)y * out_stride, src + (size_t)y * W, 2 * (size_t)W);
            }
            t_unpack += now() - t1;
            advance(unpacked, j + 1);
        }
    }

    int inputs(int f0, int nf) override
    {
        // every launch issued so far has read the inputs of the frames before f0
        for (int j = consumed; j < f0; j++) {
            hipError_t e = hipEventRecord(ev_free[j % ring], h->stream);
            if (e != hipSuccess) return hip_error(e, "hipEventRecord");
        }
        consumed = std::max(consumed, f0);
        for (int j = f0; j < f0 + nf; j++) {
            const double t0 = now();
            if (!wait_for([&] { return packed > j; })) return err ? err : SGM_ERR_DEVICE;
            const double t1 = now();
            t_drv_in += t1 - t0;
            const int slot = j % ring;
            hipError_t e = hipSuccess;
            if (j >= ring) e = hipStreamWaitEvent(h->up, ev_free[slot], 0);   // device slot read by its census
            if (e == hipSuccess)
                e = hipMemcpyAsync(din + (size_t)slot * 2 * WH, pin + (size_t)slot * 2 * WH, 2 * WH,
                                   hipMemcpyHostToDevice, h->up);
            if (e == hipSuccess) e = hipEventRecord(ev_h2d[slot], h->up);
            if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, ev_h2d[slot], 0);
            if (e != hipSuccess) return hip_error(e, "frame upload");
            t_api_in += now() - t1;
            advance(uploaded, j + 1);
        }
        return SGM_OK;
    }

    int outputs_free(int f0, int nf) override
    {
        const double t0 = now();
        struct Acc { double& a; double t; ~Acc() { a += now() - t; } } acc{t_api_free, t0};
        // The device slot is free once its previous frame reached the caller (the unpacker
        // saw that frame's D2H complete). A host-side wait: a stream wait on the copy
        // stream's event would block the host inside HIP until that copy is submitted.
        for (int j = std::max(f0, ring); j < f0 + nf; j++) {
            if (d2h_issued <= j - ring) { set_error(SGM_ERR_ARG, "output ring overrun"); return SGM_ERR_ARG; }
            if (!wait_for([&] { return unpacked > j - ring; })) return err ? err : SGM_ERR_DEVICE;
        }
        return SGM_OK;
    }

    int outputs_done(int f0, int nf) override
    {
        hipError_t e = hipEventRecord(ev_ready, h->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(h->down, ev_ready, 0);
        if (e != hipSuccess) return hip_error(e, "output event");
        for (int j = f0; j < f0 + nf; j++) {
            const int slot = j % ring;
            // the pinned slot's previous frame must have reached the caller's buffer
            const double t0 = now();
            if (j >= ring && !wait_for([&] { return unpacked > j - ring; })) return err ? err : SGM_ERR_DEVICE;
            t_drv_out += now() - t0;
            const double t1 = now();
            e = hipMemcpyAsync(pout + (size_t)slot * WH, dout + (size_t)slot * WH, WH * 2, hipMemcpyDeviceToHost,
                               h->down);
            if (e == hipSuccess) e = hipEventRecord(ev_d2h[slot], h->down);
            if (e != hipSuccess) return hip_error(e, "frame download");
            t_api_out += now() - t1;
            advance(d2h_issued, j + 1);
        }
        return SGM_OK;
    }
};

// Device + pinned rings and the copy streams / events of a handle (kept across calls).
int ensure_io(sgm_handle* h, size_t WH)
{
    const int ring = io_ring_frames(WH);
    const size_t dev_bytes = align_up((size_t)ring * 2 * WH) + align_up((size_t)ring * 2 * WH);
    const size_t pin_bytes = (size_t)ring * 4 * WH;
    // copy streams at the highest priority: when a copy runs as a blit kernel, its few
    // workgroups are dispatched ahead of the pipeline launch's queued ones
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    // (-DSGM_IO_PRIO=0, a measurement build: the copy streams at the default priority)
    const int prio = SGM_IO_PRIO ? hi : 0;
    if (!h->up) HIP_TRY(hipStreamCreateWithPriority(&h->up, hipStreamNonBlocking, prio), "hipStreamCreate");
    if (!h->down) HIP_TRY(hipStreamCreateWithPriority(&h->down, hipStreamNonBlocking, prio), "hipStreamCreate");
    while (h->io_ev.size() < 3 * kIoRing + 1) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        h->io_ev.push_back(e);
    }
    if (h->io_dev_size < dev_bytes) {
        if (h->io_dev) { (void)hipFree(h->io_dev); h->io_dev = nullptr; h->io_dev_size = 0; }
        HIP_TRY(hipMalloc(&h->io_dev, dev_bytes), "hipMalloc frame ring");
        h->io_dev_size = dev_bytes;
    }
    if (h->io_pin_size < pin_bytes) {
        if (h->io_pin) { (void)hipHostFree(h->io_pin); h->io_pin = nullptr; h->io_pin_size = 0; }
        HIP_TRY(hipHostMalloc((void**)&h->io_pin, pin_bytes, hipHostMallocDefault), "hipHostMalloc frame ring");
        h->io_pin_size = pin_bytes;
    }
    return SGM_OK;
}

// The frames `idx` of a host batch on one device handle (census mode: the pipelined
// batch of run_batch_census; other modes: one pipeline per frame), streamed as above.
int stream_host_frames(sgm_handle* h, const uint8_t* const* lefts, const uint8_t* const* rights,
                       int16_t* const* disps, const std::vector<int>& idx, int W, int H, size_t stride,
                       size_t out_stride)
{
    const int n = (int)idx.size();
    if (n == 0) return SGM_OK;
    std::lock_guard<std::mutex> lk(h->mu);
    Geom g;
    int rc = make_geom(h->params, W, H, g, h->err);
    if (rc) return rc;
    const bool pipelined = h->params.mode == SGM_MODE_CENSUS8 && n >= 2 && g.width1 > 0;
    Layout l;
    if ((rc = prepare(h, W, H, false, g, l, pipelined ? batch_group(n) : 0))) return rc;
    if ((rc = order_after_last(h, h->stream))) return rc;
    const size_t WH = (size_t)W * H;
    if ((rc = ensure_io(h, WH))) return rc;
    HostStreamer s;
    s.h = h; s.W = W; s.H = H; s.stride = stride; s.out_stride = out_stride; s.WH = WH; s.n = n;
    for (int i : idx) { s.L.push_back(lefts[i]); s.R.push_back(rights[i]); s.O.push_back(disps[i]); }
    const int ring = s.ring = io_ring_frames(WH);
    s.din = (uint8_t*)h->io_dev;
    s.dout = (int16_t*)((char*)h->io_dev + align_up((size_t)ring * 2 * WH));
    s.pin = h->io_pin;
    s.pout = (int16_t*)(h->io_pin + (size_t)ring * 2 * WH);
    s.ev_h2d = h->io_ev.data();
    s.ev_free = h->io_ev.data() + kIoRing;
    s.ev_d2h = h->io_ev.data() + 2 * kIoRing;
    s.ev_ready = h->io_ev[3 * kIoRing];
    std::vector<const uint8_t*> dL(n), dR(n);
    std::vector<int16_t*> dO(n);
    for (int j = 0; j < n; j++) {
        dL[j] = s.din + (size_t)(j % ring) * 2 * WH;
        dR[j] = dL[j] + WH;
        dO[j] = s.dout + (size_t)(j % ring) * WH;
    }
    const double t_start = HostStreamer::now();
    std::thread tp([&] { s.packer(); });
    std::thread tu([&] { s.unpacker(); });
    if (pipelined) {
        rc = run_batch_census(h, l, g, dL.data(), dR.data(), n, (size_t)W, dO.data(), (size_t)W, nullptr, nullptr, 0,
                              &s);
    } else {
        for (int j = 0; j < n && !rc; j++) {
            if (!(rc = s.inputs(j, 1)) && !(rc = s.outputs_free(j, 1)) &&
                !(rc = run_pipeline(h, l, g, dL[j], dR[j], (size_t)W, dO[j], (size_t)W)))
                rc = s.outputs_done(j, 1);
        }
    }
    if (rc) {
        std::string msg = h->err;
        s.set_error(rc, msg);
    }
    const double t_end = HostStreamer::now();
    tp.join();
    tu.join();
    if (const char* tr = std::getenv("SGM_IO_TRACE"); tr && std::atoi(tr)) {
        (void)hipStreamSynchronize(h->stream);
        std::fprintf(stderr,
                     "[sgm io] dev %d frames %d: driver issue %.2f ms (waits: packed %.2f, unpacked %.2f) | packer copy %.2f "
                     "wait %.2f | unpacker copy %.2f wait %.2f | api h2d %.2f free %.2f d2h %.2f | total %.2f ms\n",
                     h->device, n, (t_end - t_start) * 1e3, s.t_drv_in * 1e3, s.t_drv_out * 1e3, s.t_pack * 1e3,
                     s.t_pack_wait * 1e3, s.t_unpack * 1e3, s.t_unpack_wait * 1e3, s.t_api_in * 1e3, s.t_api_free * 1e3,
                     s.t_api_out * 1e3, (HostStreamer::now() - t_start) * 1e3);
    }
    const hipError_t e1 = hipStreamSynchronize(h->stream), e2 = hipStreamSynchronize(h->up),
                     e3 = hipStreamSynchronize(h->down);
    if (s.err) return fail(h, s.err, s.err_msg.empty() ? h->err : s.err_msg);
    if (e1 != hipSuccess) return hip_fail(h, e1, "hipStreamSynchronize");
    if (e2 != hipSuccess) return hip_fail(h, e2, "hipStreamSynchronize up");
    if (e3 != hipSuccess) return hip_fail(h, e3, "hipStreamSynchronize down");
    return mark_done(h, h->stream);
}

}  // namespace

extern "C" {

int sgm_match_batch(sgm_handle* h, const uint8_t* const* lefts, const uint8_t* const* rights, int n_frames, int W,
                    int H, size_t stride, int16_t* const* disps, size_t out_stride, const int* devices, int n_dev)
{
    if (!h || !lefts || !rights || !disps || n_frames < 0) return SGM_ERR_ARG;
    if (W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W) return fail(h, SGM_ERR_ARG, "bad sizes");
    for (int i = 0; i < n_frames; i++)
        if (!lefts[i] || !rights[i] || !disps[i]) return fail(h, SGM_ERR_ARG, "null frame pointer");
    if (n_frames == 0) return SGM_OK;
    std::vector<int> devs;
    int rc = open_subs(h, devices, n_dev, devs);
    if (rc) return rc;
    const int nd = (int)devs.size();
    return run_on_subs(h, devs, [&](int t, sgm_handle* sub) {
        std::vector<int> mine;
        for (int i = t; i < n_frames; i += nd) mine.push_back(i);
        return stream_host_frames(sub, lefts, rights, disps, mine, W, H, stride, out_stride);
    });
}

int sgm_match_tiled(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, int16_t* disp,
                    size_t out_stride, int n_bands, int halo, const int* devices, int n_dev)
{
    if (!h) return SGM_ERR_ARG;
    if (!L || !R || !disp || W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W || n_bands < 1 ||
        halo < 0)
        return fail(h, SGM_ERR_ARG, "bad buffers, sizes, band count or halo");
    n_bands = std::min(n_bands, H);
    std::vector<int> devs;
    int rc = open_subs(h, devices, n_dev, devs);
    if (rc) return rc;
    const int nd = (int)devs.size();
    return run_on_subs(h, devs, [&](int t, sgm_handle* sub) {
        std::vector<int16_t> band;
        for (int b = t; b < n_bands; b += nd) {
            const int c0 = (int)((long long)b * H / n_bands), c1 = (int)((long long)(b + 1) * H / n_bands);
            const int e0 = std::max(0, c0 - halo), e1 = std::min(H, c1 + halo);
            band.resize((size_t)W * (e1 - e0));
            int r = sgm_match(sub, L + (size_t)e0 * stride, R + (size_t)e0 * stride, W, e1 - e0, stride, band.data(),
                              (size_t)W);
            if (r) return r;
            for (int y = c0; y < c1; y++)
                std::memcpy(disp + (size_t)y * out_stride, band.data() + (size_t)(y - e0) * W, sizeof(int16_t) * W);
        }
        return (int)SGM_OK;
    });
}

}  // extern "C"

static bool enable_peer_pair(int a, int b);

// Overlap tile mode on device buffers (the C5 frame already in HBM of h's device): band b's
// rows + halo go device -> devices[b % n] (xGMI peer copy), are matched there by
// sgm_match_device on that device's sub-handle, and the band's own rows come back into
// d_disp. Each device's bands run on its own host thread and stream.
static int tiled_copy(void* dst, int ddev, size_t dpitch, const void* src, int sdev, size_t spitch, size_t width,
                      size_t rows, bool peer_ok, hipStream_t st)
{
    if (ddev != sdev && dpitch == width && spitch == width) {      // contiguous rows: one peer copy
        const hipError_t e = hipMemcpyPeerAsync(dst, ddev, src, sdev, width * rows, st);
        return e == hipSuccess ? 0 : (int)e;
    }
    // strided rows within a device, or between devices whose peer access is confirmed both ways
    // (enable_peer_pair): one 2-D copy over the unified address space. Peer copies between
    // devices without peer mappings take one hipMemcpyPeerAsync per row (the runtime stages them).
    // (Between distinct physical devices this path has not run on hardware: the leased boxes have
    // one GPU)
    if (ddev == sdev || peer_ok) {
        const hipError_t e = hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDefault, st);
        if (e == hipSuccess) return 0;
        if (ddev == sdev) return (int)e;
        (void)hipGetLastError();
    }
    for (size_t r = 0; r < rows; r++) {
        const hipError_t e2 = hipMemcpyPeerAsync((char*)dst + r * dpitch, ddev, (const char*)src + r * spitch, sdev,
                                                 width, st);
        if (e2 != hipSuccess) return (int)e2;
    }
    return 0;
}

extern "C" int sgm_match_tiled_device(sgm_handle* h, const uint8_t* dL, const uint8_t* dR, int W, int H,
                                      size_t stride, int16_t* dOut, size_t out_stride, int n_bands, int halo,
                                      const int* devices, int n_dev, void* stream)
{
    if (!h) return SGM_ERR_ARG;
    if (!dL || !dR || !dOut || W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W || n_bands < 1 ||
        halo < 0)
        return fail(h, SGM_ERR_ARG, "bad buffers, sizes, band count or halo");
    if (h->rect_on) return fail(h, SGM_ERR_UNSUPPORTED, "the tile mode takes rectified images");
    n_bands = std::min(n_bands, H);
    std::vector<int> devs;
    int rc = open_subs(h, devices, n_dev, devs);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        if ((rc = ensure_stream(h))) return rc;
        if (stream) HIP_TRY(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize caller");
        if (h->done_stream) HIP_TRY(hipEventSynchronize(h->done), "hipEventSynchronize");
    }
    std::vector<char> peer_ok(devs.size(), 0);           // peer access confirmed both ways
    for (size_t i = 0; i < devs.size(); i++) peer_ok[i] = enable_peer_pair(devs[i], h->device) ? 1 : 0;
    const int nd = (int)devs.size(), hdev = h->device;
    return run_on_subs(h, devs, [&](int t, sgm_handle* sub) {
        for (int b = t; b < n_bands; b += nd) {
            const int c0 = (int)((long long)b * H / n_bands), c1 = (int)((long long)(b + 1) * H / n_bands);
            const int e0 = std::max(0, c0 - halo), e1 = std::min(H, c1 + halo), He = e1 - e0;
            const size_t img = align_up((size_t)W * He), need = 2 * img + (size_t)W * He * 2;
            int r = ensure_stream(sub);
            if (r) return r;
            if (sub->io_dev_size < need) {
                (void)hipStreamSynchronize(sub->stream);
                if (sub->io_dev) { (void)hipFree(sub->io_dev); sub->io_dev = nullptr; sub->io_dev_size = 0; }
                if (hipMalloc(&sub->io_dev, need) != hipSuccess)
                    return fail(sub, SGM_ERR_ALLOC, "hipMalloc band buffers");
                sub->io_dev_size = need;
            }
            uint8_t* bl = (uint8_t*)sub->io_dev;
            uint8_t* br = bl + img;
            int16_t* bo = (int16_t*)(br + img);
            const bool pk = peer_ok[t] != 0;
            if ((r = tiled_copy(bl, sub->device, W, dL + (size_t)e0 * stride, hdev, stride, W, He, pk, sub->stream)) ||
                (r = tiled_copy(br, sub->device, W, dR + (size_t)e0 * stride, hdev, stride, W, He, pk, sub->stream)))
                return fail(sub, SGM_ERR_DEVICE, std::string("band input copy: ") + hipGetErrorString((hipError_t)r));
            if ((r = sgm_match_device(sub, bl, br, W, He, W, bo, W, nullptr))) return r;
            if ((r = tiled_copy(dOut + (size_t)c0 * out_stride, hdev, out_stride * 2, bo + (size_t)(c0 - e0) * W,
                                sub->device, (size_t)W * 2, (size_t)W * 2, c1 - c0, pk, sub->stream)))
                return fail(sub, SGM_ERR_DEVICE, std::string("band output copy: ") + hipGetErrorString((hipError_t)r));
            if (hipStreamSynchronize(sub->stream) != hipSuccess) return fail(sub, SGM_ERR_DEVICE, "band stream");
        }
        return (int)SGM_OK;
    });
}

// ------------------------------------------------------------------ exact tile mode ----
// SURVEY §8(e) "single huge frame", exact mode. Band b (rows [c0, c1)) runs on its own
// handle: census of its rows (+3 image rows of halo, so the codes equal the full frame's),
// horizontal scans (band-local), then its downward sweeps continue the lines of band b-1
// from band b-1's last volume row and its upward sweeps those of band b+1 from its first
// row. The boundary rows (3 directions x width1 x D u8 per seam and sweep) move between
// devices with hipMemcpyPeerAsync (xGMI); the two chains run top-down and bottom-up
// concurrently (separate streams), so the frame's critical path is H row steps per sweep
// direction, whatever the band count. The WTA of a band needs only its own rows.
namespace {

constexpr unsigned kDirsHoriz = 0xC0u, kDirsDown = 0x0Du, kDirsUp = 0x32u;

struct BandLayout {
    size_t inL = 0, inR = 0, cL = 0, cR = 0, vols = 0, vol_bytes = 0, items[3] = {}, bnd[2] = {}, bnd_slot = 0, raw = 0;
    int n_items[3] = {};
    size_t total = 0;
};

BandLayout make_band_layout(const Geom& g, int He)
{
    BandLayout l;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + std::max<size_t>(bytes, 1)); return o; };
    const size_t w1 = (size_t)std::max(g.width1, 0);    // width1 <= 0: no paths, all invalid
    const size_t cells = w1 * g.H * g.D;
    l.inL = take((size_t)g.W * He);
    l.inR = take((size_t)g.W * He);
    auto take_codes = [&](size_t n) { return take((n + 2 * sgm::kCodeMargin) * 8) + 8 * sgm::kCodeMargin; };
    l.cL = take_codes((size_t)g.W * He);
    l.cR = take_codes((size_t)g.W * He);
    l.vol_bytes = align_up(cells + kTrashBytes);
    l.vols = take(l.vol_bytes * 8);
    const unsigned masks[3] = {kDirsHoriz, kDirsDown, kDirsUp};
    for (int i = 0; i < 3; i++) {
        l.n_items[i] = w1 ? sgm::census_path_items(g, masks[i], 1, 1, nullptr, 0) : 0;
        l.items[i] = take((size_t)l.n_items[i] * 4);
    }
    // + 512 B: lanes past D (D < 16 * DPL) read beyond the last pixel before being masked
    l.bnd_slot = align_up(w1 * g.D + 512);
    l.bnd[0] = take(3 * l.bnd_slot);
    l.bnd[1] = take(3 * l.bnd_slot);
    l.raw = take((size_t)g.W * g.H * 2);
    l.total = off;
    return l;
}

hipError_t copy_between(void* dst, int ddev, const void* src, int sdev, size_t n, hipStream_t st)
{
    return ddev == sdev ? hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st)
                        : hipMemcpyPeerAsync(dst, ddev, src, sdev, n, st);
}

// Enables dev -> peer access; true when it is in effect (enabled now or before, or dev == peer).
bool enable_peer(int dev, int peer)
{
    if (dev == peer) return true;
    int ok = 0;
    if (hipDeviceCanAccessPeer(&ok, dev, peer) != hipSuccess || !ok) {
        (void)hipGetLastError();
        return false;
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(dev) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    (void)hipGetLastError();
    if (prev >= 0) (void)hipSetDevice(prev);
    return e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
}

// Stream 2 + events of a band handle; the three path work lists uploaded for g.
int band_prepare(sgm_handle* b, const Geom& g, const BandLayout& l)
{
    sgm_handle* h = b;                            // for HIP_TRY
    int rc = ensure_stream(b);
    if (rc) return rc;
    if (!b->stream2) HIP_TRY(hipStreamCreateWithFlags(&b->stream2, hipStreamNonBlocking), "hipStreamCreate");
    for (hipEvent_t& e : b->bev)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    if ((rc = ensure_ws(b, l.total))) return rc;
    char key[160];
    snprintf(key, sizeof key, "band %d %d %d %d %d %zu %p", g.W, g.H, g.D, g.minD, b->n_cu, l.total, b->ws.base);
    if (b->items_key[0] == key) return SGM_OK;
    const unsigned masks[3] = {kDirsHoriz, kDirsDown, kDirsUp};
    std::vector<uint32_t> v;
    for (int i = 0; i < 3 && g.width1 > 0; i++) {
        const int n = sgm::census_path_items(g, masks[i], b->n_cu, 1, nullptr, 0);
        if (n != l.n_items[i]) return fail(b, SGM_ERR_ARG, "band work list size mismatch");
        v.resize(n);
        sgm::census_path_items(g, masks[i], b->n_cu, 1, v.data(), n);
        HIP_TRY(hipMemcpy((char*)b->ws.base + l.items[i], v.data(), (size_t)n * 4, hipMemcpyHostToDevice), "H2D items");
    }
    b->items_key[0] = key;
    b->items_key[1].clear();
    return SGM_OK;
}

// Post-filter workspace of the assembled frame on the primary handle.
Layout make_post_layout(const sgm_params& p, const Geom& g)
{
    Layout l;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + std::max<size_t>(bytes, 1)); return o; };
    const size_t WH = (size_t)g.W * g.H;
    l.tmp = take(WH * 2);
    l.out = take(WH * 2);
    if (p.speckle_window_size > 0) { l.lab = take(WH * 4); l.cnt = take(WH * 4); }
    l.total = off;
    return l;
}

int run_tiled_exact(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, int16_t* disp,
                    size_t out_stride, int n_bands, const std::vector<int>& devs)
{
    const sgm_params& p = h->params;
    Geom gf;
    int rc = make_geom(p, W, H, gf, h->err);
    if (rc) return rc;
    if (p.mode != SGM_MODE_CENSUS8) return fail(h, SGM_ERR_UNSUPPORTED, "the exact tile mode runs in the census mode");
    const int nb = n_bands;
    while ((int)h->bands.size() < nb) h->bands.push_back(nullptr);
    std::vector<int> c(nb + 1);
    for (int b = 0; b <= nb; b++) c[b] = (int)((long long)b * H / nb);
    std::vector<Geom> g(nb);
    std::vector<BandLayout> bl(nb);
    for (int b = 0; b < nb; b++) {
        const int dev = devs[b % devs.size()];
        sgm_handle*& bh = h->bands[b];
        if (bh && bh->device != dev) { sgm_destroy(bh); bh = nullptr; }
        if (!bh && (rc = sgm_create(&bh, dev))) return fail(h, rc, "cannot open device " + std::to_string(dev));
        bh->params = p;
        if ((rc = make_geom(p, W, c[b + 1] - c[b], g[b], h->err))) return rc;
        const int e0 = std::max(0, c[b] - 3), e1 = std::min(H, c[b + 1] + 3);
        bl[b] = make_band_layout(g[b], e1 - e0);
        if ((rc = band_prepare(bh, g[b], bl[b]))) return fail(h, rc, "band " + std::to_string(b) + ": " + bh->err);
        if ((rc = ensure_pin(bh, 2 * (size_t)W * (e1 - e0)))) return fail(h, rc, bh->err);
    }
    for (int b = 0; b < nb; b++) {
        if (b > 0) enable_peer(h->bands[b]->device, h->bands[b - 1]->device);
        if (b + 1 < nb) enable_peer(h->bands[b]->device, h->bands[b + 1]->device);
        enable_peer(h->bands[b]->device, h->device);
    }
    if ((rc = ensure_stream(h))) return rc;
    const Layout pl = make_post_layout(p, gf);
    if ((rc = ensure_ws(h, pl.total))) return rc;
    if ((rc = ensure_pin(h, (size_t)W * H * 2))) return rc;
    const bool med = use_median(p);
    char* pws = (char*)h->ws.base;
    int16_t* frame_raw = (int16_t*)(pws + (med ? pl.tmp : pl.out));
    const size_t cells_row = (size_t)std::max(gf.width1, 0) * gf.D;

    auto ws = [&](int b, size_t off) { return (char*)h->bands[b]->ws.base + off; };
    auto fail_band = [&](int b, hipError_t e, const char* where) {
        for (sgm_handle* s : h->bands)
            if (s && s->stream) { (void)hipSetDevice(s->device); (void)hipStreamSynchronize(s->stream);
                                   (void)hipStreamSynchronize(s->stream2); }
        return fail(h, SGM_ERR_DEVICE, "band " + std::to_string(b) + " " + where + ": " + hipGetErrorString(e));
    };
#define BAND_TRY(b, expr, where)                          \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return fail_band(b, e_, where); \
    } while (0)
    enum { EV_CENSUS = 0, EV_DOWN = 1, EV_UP = 2, EV_GATHER = 3 };
    // SGM_TILE_TIMES=<file>: measurement mode — every band step runs alone (synchronised
    // before and after) and its duration on the band's device is appended to the file as
    // "band kind ms" lines (the per-band inputs of the multi-device critical-path model in
    // DESIGN.md §7). Never set in production runs.
    struct TileTimes {           // closed / destroyed on every return path
        FILE* f = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~TileTimes() {
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
            if (f) std::fclose(f);
        }
    } tt;
    if (const char* tf = std::getenv("SGM_TILE_TIMES")) tt.f = std::fopen(tf, "a");
    FILE*& tt_file = tt.f;
    hipEvent_t& tt0 = tt.e0;
    hipEvent_t& tt1 = tt.e1;
    auto tt_begin = [&](int b, hipStream_t s) {
        if (!tt_file) return;
        (void)hipSetDevice(h->bands[b]->device);
        (void)hipDeviceSynchronize();
        if (!tt0) { (void)hipEventCreate(&tt0); (void)hipEventCreate(&tt1); }
        (void)hipEventRecord(tt0, s);
    };
    auto tt_end = [&](int b, const char* kind, hipStream_t s) {
        if (!tt_file) return;
        float ms = 0.f;
        (void)hipEventRecord(tt1, s);
        (void)hipEventSynchronize(tt1);
        (void)hipEventElapsedTime(&ms, tt0, tt1);
        std::fprintf(tt_file, "%d %s %.4f\n", b, kind, ms);
    };
    // 1. inputs, census, horizontal scans (band-local)
    for (int b = 0; b < nb; b++) {
        sgm_handle* bh = h->bands[b];
        BAND_TRY(b, hipSetDevice(bh->device), "hipSetDevice");
        const int e0 = std::max(0, c[b] - 3), e1 = std::min(H, c[b + 1] + 3), He = e1 - e0;
        const size_t n = (size_t)W * He;
        for (int y = 0; y < He; y++) {
            std::memcpy(bh->pin + (size_t)y * W, L + (size_t)(e0 + y) * stride, W);
            std::memcpy(bh->pin + n + (size_t)y * W, R + (size_t)(e0 + y) * stride, W);
        }
        tt_begin(b, bh->stream);
        BAND_TRY(b, hipMemcpyAsync(ws(b, bl[b].inL), bh->pin, n, hipMemcpyHostToDevice, bh->stream), "H2D");
        BAND_TRY(b, hipMemcpyAsync(ws(b, bl[b].inR), bh->pin + n, n, hipMemcpyHostToDevice, bh->stream), "H2D");
        tt_end(b, "h2d", bh->stream);
        tt_begin(b, bh->stream);
        BAND_TRY(b, sgm::launch_census((const uint8_t*)ws(b, bl[b].inL), (const uint8_t*)ws(b, bl[b].inR), W, W, He,
                                       (uint64_t*)ws(b, bl[b].cL), (uint64_t*)ws(b, bl[b].cR), bh->stream), "census");
        tt_end(b, "census", bh->stream);
        BAND_TRY(b, hipEventRecord(bh->bev[EV_CENSUS], bh->stream), "event");
    }
    auto frames = [&](int b) {
        sgm::PathFrames pf{};
        const size_t skip = (size_t)(c[b] - std::max(0, c[b] - 3)) * W;   // codes of the band's first row
        pf.cL[0] = (const uint64_t*)ws(b, bl[b].cL) + skip;
        pf.cR[0] = (const uint64_t*)ws(b, bl[b].cR) + skip;
        pf.vols[0] = (uint8_t*)ws(b, bl[b].vols);
        pf.n = 1;
        return pf;
    };
    if (gf.width1 > 0) {
        for (int b = 0; b < nb; b++) {
            sgm_handle* bh = h->bands[b];
            BAND_TRY(b, hipSetDevice(bh->device), "hipSetDevice");
            tt_begin(b, bh->stream);
            BAND_TRY(b, sgm::launch_census_paths(frames(b), bl[b].vol_bytes, g[b], (const uint32_t*)ws(b, bl[b].items[0]),
                                                 bl[b].n_items[0], bh->stream), "horizontal paths");
            tt_end(b, "horiz", bh->stream);
        }
        // 2. downward chain, top to bottom: band b continues band b-1's last row
        static const int down_dirs[3] = {0, 2, 3}, up_dirs[3] = {1, 4, 5};
        for (int b = 0; b < nb; b++) {
            sgm_handle* bh = h->bands[b];
            BAND_TRY(b, hipSetDevice(bh->device), "hipSetDevice");
            if (b > 0) BAND_TRY(b, hipStreamWaitEvent(bh->stream, h->bands[b - 1]->bev[EV_DOWN], 0), "wait");
            tt_begin(b, bh->stream);
            BAND_TRY(b, sgm::launch_census_paths(frames(b), bl[b].vol_bytes, g[b], (const uint32_t*)ws(b, bl[b].items[1]),
                                                 bl[b].n_items[1], bh->stream,
                                                 b > 0 ? (const uint8_t*)ws(b, bl[b].bnd[0]) : nullptr, nullptr,
                                                 bl[b].bnd_slot), "down paths");
            tt_end(b, "down", bh->stream);
            if (b + 1 < nb) {
                tt_begin(b, bh->stream);
                const size_t last = (size_t)(g[b].H - 1) * cells_row;
                for (int k = 0; k < 3; k++)
                    BAND_TRY(b, copy_between(ws(b + 1, bl[b + 1].bnd[0] + k * bl[b + 1].bnd_slot), h->bands[b + 1]->device,
                                             ws(b, bl[b].vols + down_dirs[k] * bl[b].vol_bytes + last), bh->device,
                                             cells_row, bh->stream), "boundary copy");
                tt_end(b, "copy_down", bh->stream);
            }
            BAND_TRY(b, hipEventRecord(bh->bev[EV_DOWN], bh->stream), "event");
        }
        // 3. upward chain, bottom to top, on the second streams: band b continues band b+1's first row
        for (int b = nb - 1; b >= 0; b--) {
            sgm_handle* bh = h->bands[b];
            BAND_TRY(b, hipSetDevice(bh->device), "hipSetDevice");
            BAND_TRY(b, hipStreamWaitEvent(bh->stream2, bh->bev[EV_CENSUS], 0), "wait");
            if (b + 1 < nb) BAND_TRY(b, hipStreamWaitEvent(bh->stream2, h->bands[b + 1]->bev[EV_UP], 0), "wait");
            tt_begin(b, bh->stream2);
            BAND_TRY(b, sgm::launch_census_paths(frames(b), bl[b].vol_bytes, g[b], (const uint32_t*)ws(b, bl[b].items[2]),
                                                 bl[b].n_items[2], bh->stream2, nullptr,
                                                 b + 1 < nb ? (const uint8_t*)ws(b, bl[b].bnd[1]) : nullptr,
                                                 bl[b].bnd_slot), "up paths");
            tt_end(b, "up", bh->stream2);
            if (b > 0) {
                tt_begin(b, bh->stream2);
                for (int k = 0; k < 3; k++)
                    BAND_TRY(b, copy_between(ws(b - 1, bl[b - 1].bnd[1] + k * bl[b - 1].bnd_slot), h->bands[b - 1]->device,
                                             ws(b, bl[b].vols + up_dirs[k] * bl[b].vol_bytes), bh->device, cells_row,
                                             bh->stream2), "boundary copy");
                tt_end(b, "copy_up", bh->stream2);
            }
            BAND_TRY(b, hipEventRecord(bh->bev[EV_UP], bh->stream2), "event");
        }
    }
    // 4. WTA of each band (after its three path launches), gathered into the primary's frame
    for (int b = 0; b < nb; b++) {
        sgm_handle* bh = h->bands[b];
        BAND_TRY(b, hipSetDevice(bh->device), "hipSetDevice");
        int16_t* raw = (int16_t*)ws(b, bl[b].raw);
        if (gf.width1 > 0) {
            BAND_TRY(b, hipStreamWaitEvent(bh->stream, bh->bev[EV_UP], 0), "wait");
            sgm::WtaFrames wf{};
            wf.vols[0] = (const uint8_t*)ws(b, bl[b].vols); wf.out[0] = raw; wf.n = 1;
            tt_begin(b, bh->stream);
            BAND_TRY(b, sgm::launch_census_wta(wf, bl[b].vol_bytes, g[b], W, bh->stream), "wta");
            tt_end(b, "wta", bh->stream);
        } else {
            BAND_TRY(b, sgm::launch_fill16(raw, W, W, g[b].H, gf.invalid, bh->stream), "fill");
        }
        tt_begin(b, bh->stream);
        BAND_TRY(b, copy_between(frame_raw + (size_t)c[b] * W, h->device, raw, bh->device, (size_t)W * g[b].H * 2,
                                 bh->stream), "gather");
        tt_end(b, "gather", bh->stream);
        BAND_TRY(b, hipEventRecord(bh->bev[EV_GATHER], bh->stream), "event");
    }
#undef BAND_TRY
    // 5. post filters on the assembled frame (median / speckles need no band seams), D2H
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    for (int b = 0; b < nb; b++) HIP_TRY(hipStreamWaitEvent(h->stream, h->bands[b]->bev[EV_GATHER], 0), "wait");
    StageRec rec{h};
    int16_t* out = (int16_t*)(pws + pl.out);
    if (tt_file) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(tt0, h->stream);
    }
    if ((rc = run_post(h, pl, gf, out, W, rec))) return rc;
    rec.end();
    if (tt_file) {
        float ms = 0.f;
        (void)hipEventRecord(tt1, h->stream);
        (void)hipEventSynchronize(tt1);
        (void)hipEventElapsedTime(&ms, tt0, tt1);
        std::fprintf(tt_file, "-1 post %.4f\n", ms);
    }
    HIP_TRY(hipMemcpyAsync(h->pin, out, (size_t)W * H * 2, hipMemcpyDeviceToHost, h->stream), "D2H");
    HIP_TRY(hipStreamSynchronize(h->stream), "sync");
    const int16_t* src = (const int16_t*)h->pin;
    for (int y = 0; y < H; y++) std::memcpy(disp + (size_t)y * out_stride, src + (size_t)y * W, 2 * (size_t)W);
    return SGM_OK;
}

}  // namespace

static bool enable_peer_pair(int a, int b)
{
    const bool ab = enable_peer(a, b), ba = enable_peer(b, a);
    return ab && ba;
}

extern "C" {

int sgm_match_tiled_exact(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride,
                          int16_t* disp, size_t out_stride, int n_bands, const int* devices, int n_dev)
{
    if (!h) return SGM_ERR_ARG;
    if (!L || !R || !disp || W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W || n_bands < 1)
        return fail(h, SGM_ERR_ARG, "bad buffers, sizes or band count");
    std::vector<int> devs;
    if (!devices || n_dev <= 0) {
        for (int i = 0; i < sgm_device_count(); i++) devs.push_back(i);
    } else {
        devs.assign(devices, devices + n_dev);
    }
    if (devs.empty()) return fail(h, SGM_ERR_DEVICE, "no HIP device");
    std::lock_guard<std::mutex> lk(h->mu);
    return run_tiled_exact(h, L, R, W, H, stride, disp, out_stride, std::min(n_bands, H), devs);
}

int sgm_set_profiling(sgm_handle* h, int enable)
{
    if (!h) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    h->profiling = enable != 0;
    h->ev_used = 0;
    h->launches.clear();
    h->prof_frames = 0;
    h->nstages = 0;
    return SGM_OK;
}

int sgm_profiled_matches(const sgm_handle* h) { return h ? h->prof_frames : 0; }

int sgm_get_stage_times(sgm_handle* h, float* ms, int max)
{
    if (!h || !ms) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->launches.empty()) return 0;
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    HIP_TRY(hipEventSynchronize(h->ev_pool[h->ev_used - 1]), "hipEventSynchronize");
    const int n = std::min(h->nstages, max);
    std::vector<double> acc(h->nstages, 0.0);
    std::vector<int> cnt(h->nstages, 0);
    for (const auto& r : h->launches) {
        if (r.ev1 == r.ev0) continue;           // never closed
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, h->ev_pool[r.ev0], h->ev_pool[r.ev1]), "hipEventElapsedTime");
        acc[r.stage] += t;
        cnt[r.stage]++;
    }
    for (int i = 0; i < n; i++) ms[i] = (float)(acc[i] / std::max(cnt[i], 1));
    return n;
}

const char* sgm_stage_name(const sgm_handle* h, int i)
{
    if (!h || i < 0 || i >= h->nstages) return "";
    return h->stage_name[i];
}

double sgm_stage_bytes(const sgm_handle* h, int i)
{
    if (!h || i < 0 || i >= h->nstages) return 0.0;
    return h->stage_bytes[i];
}

int sgm_stage_launches(const sgm_handle* h, int i)
{
    if (!h || i < 0 || i >= h->nstages) return 0;
    int c = 0;
    for (const auto& r : h->launches) c += (r.stage == i && r.ev1 != r.ev0) ? 1 : 0;
    return c;
}

// ------------------------------------------------------------------ stage entry points
int sgm_debug_census(sgm_handle* h, const uint8_t* img, int W, int H, size_t stride, uint64_t* out)
{
    if (!h || !img || !out || W <= 0 || H <= 0 || stride < (size_t)W) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure_stream(h);
    if (rc || (rc = order_after_last(h, h->stream))) return rc;
    const size_t WH = (size_t)W * H;
    if ((rc = ensure_ws(h, align_up(WH) + WH * 8))) return rc;
    char* ws = (char*)h->ws.base;
    HIP_TRY(hipMemcpy2DAsync(ws, W, img, stride, W, H, hipMemcpyHostToDevice, h->stream), "H2D");
    HIP_TRY(sgm::launch_census((const uint8_t*)ws, nullptr, W, W, H, (uint64_t*)(ws + align_up(WH)), nullptr,
                               h->stream), "census");
    HIP_TRY(hipMemcpyAsync(out, ws + align_up(WH), WH * 8, hipMemcpyDeviceToHost, h->stream), "D2H");
    HIP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SGM_OK;
}

int sgm_debug_census_path(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, int dir,
                          uint8_t* vol)
{
    if (!h || !L || !R || !vol || dir < 0 || dir > 7) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->params.mode != SGM_MODE_CENSUS8) return fail(h, SGM_ERR_PARAM, "census mode required");
    Geom g;
    Layout l;
    int rc = prepare(h, W, H, true, g, l);
    if (rc || (rc = order_after_last(h, h->stream))) return rc;
    if (g.width1 <= 0) return SGM_OK;
    char* ws = (char*)h->ws.base;
    HIP_TRY(hipMemcpy2DAsync(ws + l.inL, W, L, stride, W, H, hipMemcpyHostToDevice, h->stream), "H2D");
    HIP_TRY(hipMemcpy2DAsync(ws + l.inR, W, R, stride, W, H, hipMemcpyHostToDevice, h->stream), "H2D");
    uint64_t* cL = (uint64_t*)(ws + l.cL[0]);
    uint64_t* cR = (uint64_t*)(ws + l.cR[0]);
    uint8_t* vols = (uint8_t*)(ws + l.vols[0]);
    HIP_TRY(sgm::launch_census((const uint8_t*)(ws + l.inL), (const uint8_t*)(ws + l.inR), W, W, H, cL, cR, h->stream),
            "census");
    const uint32_t* items;
    const int n_items = path_items(h, l, g, 1u << dir, 1, h->stream, &items);
    if (n_items < 0) return n_items;
    sgm::PathFrames pf{};
    pf.cL[0] = cL; pf.cR[0] = cR; pf.vols[0] = vols; pf.n = 1;
    HIP_TRY(sgm::launch_census_paths(pf, l.vol_bytes, g, items, n_items, h->stream), "paths");
    const size_t cells = (size_t)g.width1 * g.H * g.D;
    HIP_TRY(hipMemcpyAsync(vol, vols + (size_t)dir * l.vol_bytes, cells, hipMemcpyDeviceToHost, h->stream), "D2H");
    HIP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SGM_OK;
}

int sgm_debug_ocv_cost(sgm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, size_t stride, int16_t* cost)
{
    if (!h || !L || !R || !cost) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->params.mode == SGM_MODE_CENSUS8) return fail(h, SGM_ERR_PARAM, "OCV mode required");
    Geom g;
    Layout l;
    int rc = prepare(h, W, H, true, g, l);
    if (rc || (rc = order_after_last(h, h->stream))) return rc;
    if (g.width1 <= 0) return SGM_OK;
    char* ws = (char*)h->ws.base;
    HIP_TRY(hipMemcpy2DAsync(ws + l.inL, W, L, stride, W, H, hipMemcpyHostToDevice, h->stream), "H2D");
    HIP_TRY(hipMemcpy2DAsync(ws + l.inR, W, R, stride, W, H, hipMemcpyHostToDevice, h->stream), "H2D");
    int16_t* A = (int16_t*)(ws + l.bufA);
    int16_t* B = (int16_t*)(ws + l.bufB);
    int flag = 0;
    if (g.wide == 2) {
        g.ovf = (int*)(ws + l.ovf);
        HIP_TRY(hipMemsetAsync(g.ovf, 0, sizeof(int), h->stream), "hipMemsetAsync");
    }
    HIP_TRY(sgm::launch_ocv_cost((const uint8_t*)(ws + l.inL), (const uint8_t*)(ws + l.inR), W, g,
                                 h->params.mode == SGM_MODE_OCV_HH8, (uint8_t*)(ws + l.planes), A, B, h->stream),
            "ocv_cost");
    if (g.wide == 2) HIP_TRY(hipMemcpyAsync(&flag, g.ovf, sizeof(int), hipMemcpyDeviceToHost, h->stream), "D2H flag");
    HIP_TRY(hipStreamSynchronize(h->stream), "sync");
    // C' of every frame kind ends in bufA (SIMD_SAT frames in the overflow regime: the exact
    // saturating cost, written over the plain one)
    (void)flag;
    const size_t cells = (size_t)g.width1 * g.H * g.D;
    HIP_TRY(hipMemcpyAsync(cost, A, cells * 2, hipMemcpyDeviceToHost, h->stream), "D2H");
    HIP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SGM_OK;
}

static int debug_post(sgm_handle* h, int16_t* disp, int W, int H, int which, int nv, int ms, int md)
{
    if (!h || !disp || W <= 0 || H <= 0) return SGM_ERR_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure_stream(h);
    if (rc || (rc = order_after_last(h, h->stream))) return rc;
    const size_t WH = (size_t)W * H;
    if ((rc = ensure_ws(h, align_up(WH * 2) * 2 + align_up(WH * 4) * 2))) return rc;
    char* ws = (char*)h->ws.base;
    int16_t* a = (int16_t*)ws;
    int16_t* b = (int16_t*)(ws + align_up(WH * 2));
    int* lab = (int*)(ws + 2 * align_up(WH * 2));
    int* cnt = (int*)(ws + 2 * align_up(WH * 2) + align_up(WH * 4));
    HIP_TRY(hipMemcpyAsync(a, disp, WH * 2, hipMemcpyHostToDevice, h->stream), "H2D");
    if (which == 0) {
        HIP_TRY(sgm::launch_median3(a, W, b, W, W, H, h->stream), "median3");
        HIP_TRY(hipMemcpyAsync(disp, b, WH * 2, hipMemcpyDeviceToHost, h->stream), "D2H");
    } else {
        HIP_TRY(sgm::launch_speckle(nullptr, 0, a, W, W, H, nv, ms, md, lab, cnt, h->stream), "speckle");
        HIP_TRY(hipMemcpyAsync(disp, a, WH * 2, hipMemcpyDeviceToHost, h->stream), "D2H");
    }
    HIP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SGM_OK;
}

int sgm_debug_median3(sgm_handle* h, int16_t* disp, int W, int H) { return debug_post(h, disp, W, H, 0, 0, 0, 0); }

int sgm_debug_path_items(const sgm_params* p, int width, int height, unsigned dir_mask, int n_slots, int group,
                         int up_group, uint32_t* out, int cap)
{
    if (!p || p->mode != SGM_MODE_CENSUS8) return SGM_ERR_ARG;
    Geom g;
    std::string err;
    const int rc = make_geom(*p, width, height, g, err);
    if (rc) return rc;
    if (g.width1 <= 0) return 0;
    const int n = sgm::census_path_items(g, dir_mask & 0xFFu, n_slots, group, nullptr, 0, up_group);
    if (!out) return n;
    if (n > cap) return SGM_ERR_ARG;
    return sgm::census_path_items(g, dir_mask & 0xFFu, n_slots, group, out, cap, up_group);
}

int sgm_debug_speckle(sgm_handle* h, int16_t* disp, int W, int H, int new_val, int max_size, int max_diff)
{
    return debug_post(h, disp, W, H, 1, new_val, max_size, max_diff);
}

}  // extern "C"
