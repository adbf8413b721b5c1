// Host/device interface of the CTC beam-search kernels (ctc_beam.hip).
#pragma once
#include "asr_internal.h"

namespace asr {

#ifdef ASR_CTC_WSTAMPS
constexpr int NSTAMP = 16 * 9;   // diagnostic: per-wave arrival clocks per utterance + critical path
#else
constexpr int NSTAMP = 16;   // diagnostic phase clocks per utterance
#endif

// Launch geometry of one decode, shared by the host planner and the kernel.
struct CtcGeom {
    int V;       // labels incl. blank (<= 63: register kernels; larger: wide kernel)
    int blank;   // blank label id
    int K;       // beamWidth + 1 states kept (cpp:107 cutoff index)
    int kcap;    // slot/state capacity incl. ties at the cutoff
    int sb;      // log2 of the candidate row stride (row = V+1 columns)
    int ch;      // emission frames staged per prefetch chunk
    int ht;      // orphan-table cells (4 x row capacity, 8-cell buckets)
    int lbits;   // bits per label in node records and tails: 8 (V <= 64) or 16
    int ts;      // timesteps mode: the workgroup kernel's TS0/TS1 arrays are allocated (Lds::total_ts)
};

struct CtcArgs {
    CtcGeom g;
    const float* emis;      // element (t, b, v) at emis[t*tstride + b*ustride + v]
    long tstride, ustride;  // time-major [T][B][V]: B*V, V; batch-major [B][T][V]: V, T*V
    const int* lengths;     // [B] frames per utterance (device; NULL = T for all)
    int T, B;
    int is_log;
    int cu_mode;            // 1: CTCBeamSearch.cu semantics (exactly beam states, strip-then-merge last)
    uint64_t blank_less;    // bit c: code(blank) < code(c)   (V <= 64 kernels)
    const int* codes;       // [V] symbol codes (device; wide-vocabulary kernel)
    int4* nodes;            // [B][T*kcap] (parent node, 0, 8 labels packed lo, hi)
    int4* nodes_ts;         // [B][T*kcap] append frames of a record's labels, 16 bits each (NULL: no timesteps)
    uint64_t* fin_ts;       // [B][kcap][2] append frames of the final tails' labels (timesteps mode)
    int* fin_n;             // [B] final hypotheses
    int* fin_node;          // [B][kcap]
    uint64_t* fin_tail;     // [B][kcap]  labels after fin_node's block (count << 56)
    double* fin_score;      // [B][kcap]
    int* status;            // [B] 1 = beam overflow
    int* best_lab;          // [B][T] reversed labels of the best hypothesis
    int* best_len;          // [B]
    double* best_score;     // [B]
    uint64_t* stamps;       // [B][NSTAMP] phase clocks (diagnostic build only)
    uint32_t* tile0;        // [B][T][WREC] first label tile per frame (wide kernel, V > 65; NULL: in-kernel)
    int tile0_ext;          // 1: the caller filled tile0 for this launch's frames (ctc_launch_tile0 on its stream)
    int diag;               // bit 0: the wide kernel always takes its register fallback (tests; ASR_CTC_WIDE_FALLBACK=1);
                            // bit 1: its adoption list holds no hit: every adoption takes the one-thread scan (tests; ASR_CTC_WIDE_ADOPT_CAP=1)
    // Segmented decode (asr_ctc_decode_segment; one-wave kernel only): this
    // launch runs frames [t0, t1) of T, emis addresses frame t0, and the beam
    // of every unfinished utterance is saved to / restored from seg_state
    // [B][seg_bytes] at the segment ends.  A whole decode: t0 = 0, t1 = T,
    // seg_state = NULL.
    int t0, t1;
    unsigned char* seg_state;
    int seg_bytes;
};

int ctc_row_capacity(int kcap);   // compile-time slot capacity KC >= kcap (64, 128, 256)
size_t ctc_lds_bytes(const CtcGeom& g);
int ctc_launch_decode_v8(const CtcArgs& a, int waves, int rpt, hipStream_t s);
int ctc_launch_decode_v32(const CtcArgs& a, int waves, int rpt, hipStream_t s);
int ctc_launch_decode_v64(const CtcArgs& a, int waves, int rpt, hipStream_t s);
int ctc_set_max_lds_v8();
int ctc_set_max_lds_v32();
int ctc_set_max_lds_v64();
int ctc_occupancy_v8(const CtcGeom& g, int waves, int rpt);
int ctc_occupancy_v32(const CtcGeom& g, int waves, int rpt);
int ctc_occupancy_v64(const CtcGeom& g, int waves, int rpt);
// Workgroups per CU of the workgroup kernel with `waves` waves (V <= 63, CPU
// semantics); 0 when that variant is not built or the query fails.
int ctc_occupancy(const CtcGeom& g, int waves);
constexpr int WIDE_VMAX = 4096;   // largest vocabulary of the wide kernel (ctc_wide_kernel.inc)
int ctc_launch_decode_wide(const CtcArgs& a, int rpt, hipStream_t s);
size_t ctc_tile0_bytes(int B, int T);   // a.tile0 workspace of the wide kernel
int ctc_launch_tile0(const CtcArgs& a, hipStream_t s);   // a.tile0 for frames [a.t0, a.t1) (a.emis at a.t0)
size_t ctc_lds_bytes_wide(int kc, int V);
size_t ctc_seg_bytes_wide(int kc);   // saved beam per utterance between segments (wide kernel)
int ctc_set_max_lds_wide();
// One wave per utterance (ctc_wave_kernel.inc): batches of many utterances per CU.
size_t ctc_lds_bytes_wave(const CtcGeom& g);
bool ctc_wave_supported(const CtcGeom& g, int cu_mode);
int ctc_launch_decode_wave(const CtcArgs& a, hipStream_t s);
int ctc_occupancy_wave(const CtcGeom& g);   // one-wave workgroups per CU
size_t ctc_seg_bytes_wave(const CtcGeom& g);  // saved beam per utterance between segments
int ctc_set_max_lds_wave();
// waves < 0: the one-wave list kernel; 1..8: the workgroup kernel with that many waves.
int ctc_launch_decode(const CtcArgs& a, int waves, hipStream_t s);
int ctc_launch_best(const CtcArgs& a, const int* d_codes, int* d_chain, hipStream_t s);
int ctc_launch_all(const CtcArgs& a, int* d_all_lab, int* d_all_len, int* d_all_ts, hipStream_t s);
int ctc_set_max_lds();

}  // namespace asr
