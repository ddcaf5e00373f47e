// transr_cons.hpp -- host entry points of the register-resident transRNorm
// kernel (kernels_transr_cons.hpp), compiled in its own translation unit
// (transr_cons.hip): one instantiation per live k-step count.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels_transr_parallel.hpp"

namespace kb2e {

constexpr int kWideMaxN = 112;  // the wide chain's W_c [n][NP + 2] + chunk buffers fit the 160 KB LDS
constexpr int kConsPpt = 1;  // transRNorm matrix partials per tile (transr_rel_rows_kernel cons_ppt)

// Does the kernel cover this width (n <= 64)?
bool cons_wave_supported(int n);
// Dynamic LDS bytes of one workgroup; raises the kernels' LDS limit to it.
size_t cons_wave_setup(int n, int St, int esize);
// One workgroup (four waves) per tile of the batch.
template <typename T>
void cons_wave_launch(const RParArgs& a, const RParBufs<T>& bf, int grid, size_t lds, hipStream_t stream);
// Phase A of the batch's tiles (projections, x, d, y; energies + hinge, or the compat
// projections for the work-vector scan), one two-wave workgroup per tile (kernels_transr_wave.hpp).
template <typename T>
void proj_wave_launch(const RParArgs& a, const RParBufs<T>& bf, int grid, hipStream_t stream);
// The tile gradient partials dW, dr (+ tile_act) of the batch, one workgroup per tile
// (kernels_transr_wave.hpp); needs bf.x, bf.d and the hinge decisions in place.
template <typename T>
void grad_wave_launch(const RParArgs& a, const RParBufs<T>& bf, int grid, hipStream_t stream);
// transRNorm per relation, pair by pair, in chunks of 32 (kernels_transr_pipe.hpp; FP64,
// n <= 64): dynamic LDS bytes (and the kernel's limit raised to it); the launch, one
// workgroup per relation of the batch (a.brel, most frequent first), each making its
// relation's pair records at the end of its chain (chain_records).
size_t cons_seq_setup(int n);
void cons_seq_launch(const RParArgs& a, const RParBufs<double>& bf, size_t lds, hipStream_t stream);
// transRNorm per relation, pair by pair, for n <= 112 (kernels_transr_chainw.hpp,
// kernels_transr_chainwp.hpp; FP64,
// any path: the VALU tile kernels at n = 100): is the width covered, its dynamic LDS
// (the limit raised to it), and the launch of the chain (one workgroup per relation
// segment of the batch) and of its pair records' kernel.
bool cons_chainw_supported(int n);
size_t cons_chainw_setup(int n);
void cons_chainw_launch(const RParArgs& a, const RParBufs<double>& bf, size_t lds, hipStream_t stream);
// transRNorm per relation, pair by pair, for FP32 tables and 112 < n <= 128
// (kernels_transr_chaing.hpp; the same model, double arithmetic, no matrix cores):
// is the width covered, its dynamic LDS (the limit raised to it), and the launch (one
// workgroup per relation, most frequent first; its pair records made in-kernel).
bool cons_chaing_supported(int n);
size_t cons_chaing_setup(int n, int esize);
template <typename T>
void cons_chaing_launch(const RParArgs& a, const RParBufs<T>& bf, size_t lds, hipStream_t stream);
// Does that chain run software-pipelined at this width (64 < n <= 100,
// kernels_transr_chainwp.hpp; KB2E_RPAR_CHAIN=lockstep: the eight-wave lockstep kernel)?
bool cons_chainw_pipelined(int n);
// The chunk kernel's counters (relations, chunks, violators, rounds, cycles sum / max,
// most chunks of a relation), reset.
void cons_seq_take_stats(unsigned long long (&st)[64]);
// Adds the kernel's round statistics (g_rpar_rounds layout) to st and resets them.
void cons_wave_take_stats(unsigned long long (&st)[16]);

// The whole PARALLEL TransR step at 128 < n <= 512, FP64 and FP32 (kernels_transr_widep.hpp,
// transr_wide.hip): matrices from global memory, CP = ceil(n / 128) element pairs a lane.
constexpr int kWideParMaxN = 512;
struct WideGeom {
    int St = 1;             // samples a tile (the tile kernel's LDS within 150 KiB)
    int chunk = 2;          // compat scan: calls a chunk
    size_t tile_lds = 0, scan_lds = 0, chain_lds = 0;
};
bool wide_par_supported(int n);
// Chooses the geometry for (n, ld, element size) and raises the kernels' LDS limits.
WideGeom wide_setup(int n, int ld, int esize);
// Phase A (reads the tables bf names): fixed energy -- the tile kernel (energies,
// hinge, directions, partials) and the pair-dedupe inserts; compat -- projections,
// the work-vector scan (scan: chunk sums, scan_pre: their prefix; work_in -> work_out)
// with the hinge, then the partials.
template <typename T>
void wide_phase_a(const RParArgs& a, const RParBufs<T>& bf, const WideGeom& g, int tgrid, double* scan,
                  double* scan_pre, const double* work_in, double* work_out, hipStream_t st);
// Phase B: relation rows, entity rows, then (constraint) transRNorm pair by pair per
// relation (wsc: a min(nr, B) x n x ld double scratch, a workgroup's W_c each) and the
// entity rows' pair records.
template <typename T>
void wide_phase_b(const RParArgs& a, const RParBufs<T>& bf, const WideGeom& g, double* wsc, bool constraint,
                  int rel_segs_max, hipStream_t st);

}  // namespace kb2e
