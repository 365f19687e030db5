/*
 * st_tuning.h - the tuning ABI of libsimilarity_transform_tuning.so: the
 * process-wide setters of the launch tables (workgroups-per-CU caps, cache
 * policies, piece tiles, the matrix-free shape) and the flat grid's testing
 * hook.  FOR TOOLS AND TESTS ONLY: the library the drop-in callers load
 * (libsimilarity_transform.so, include/similarity_transform.h) exports none
 * of these; the tuning build is the same sources compiled with
 * -DST_TUNING_ABI=1 (Makefile), so its kernels are the library's.  Every
 * setter changes a launch's shape or cache policy only: results do not
 * depend on any of them (tests/test_gpu_tuning.py).
 */
#ifndef EIGEN_VALUE_AMD_ST_TUNING_H
#define EIGEN_VALUE_AMD_ST_TUNING_H

#include "similarity_transform.h"

/* the library is built with -fvisibility=hidden: what this header declares
 * is its whole dynamic ABI */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Testing hook: the flat launches (k_flat, one workgroup per piece) spread
 * more workgroups than a dispatch's 2^32 - 1 work-items per dimension allow
 * (fp64 from 131072^2) over a 2-D grid of rows at most max_x wide; this lowers
 * max_x (rounded down to a multiple of 8, at least 8; 0 restores the
 * default, 16777208) so the 2-D form can be checked at small sizes.
 * Process-wide; returns the limit now in force.  Results do not depend on
 * it. */
unsigned int st_set_flat_grid_limit(unsigned int max_x);

/* K0's walk order in the flat form (st_rowsum_flat and the solve loops'
 * initial row sums): -1 = pieces walked from the end of the block where its
 * loads go through the caches, 0 = front to back (the library's default),
 * 1 = from the end.  Results do not depend on it (each piece's partial sum
 * and k_parts' order are fixed).  Returns the previous mode. */
int st_set_k0_reverse(int mode);

/* Workgroups per CU of the deferred flat round's launches (dtype 0 = f32,
 * 1 = f64; nontemporal = the launch form of blocks >= 2 GiB, else the cached
 * one; slot 0..4 = a read-only round with that many pending rounds, 6 =
 * a storing round; wg_per_cu 0 = uncapped, else 2..32).  The library's
 * defaults are measured (DESIGN.md §Deferred writes); this overrides one for
 * the process, for tuning tools.  Results do not depend on it.  Returns the
 * previous value, or -1 on bad arguments. */
int st_set_defer_caps(int dtype, int nontemporal, unsigned int slot,
                      unsigned int wg_per_cu);

/* Non-temporal matrix loads in the deferred flat round's launches on cached
 * fp64 blocks (below 2 GiB): bit NP (0..4) for a read-only round with NP
 * pending rounds, bit 6 for a storing round (bit 7: its stores non-temporal
 * as well), per block size class
 * (st_defer_ntload_class: 0 below 384 MiB, 1 below 640 MiB, 2 above).  The
 * library's defaults are measured (DESIGN.md §Deferred writes); this
 * overrides one for the process, for tuning tools.  Results do not depend
 * on it.  Returns the previous mask, or -1 on bad arguments. */
int st_set_defer_ntload(unsigned int size_class, unsigned int mask);

/* The deferred rounds' cache policy in general: for dtype (0 = f32, 1 = f64)
 * and size class (as st_set_every_cache: 0 below 384 MiB, 1 below 640 MiB,
 * 2 below 2 GiB - the cached form - and 3 from 2 GiB - the non-temporal
 * form), bit NP (0..4) of a read-only round with NP pending and bit 6 of a
 * storing round turn that launch's matrix loads over (cached <->
 * non-temporal), bit 7 the storing round's stores.  fp64 classes 0..2 are
 * st_set_defer_ntload's masks.  For tuning tools; results do not depend on
 * it.  Returns the previous mask, or -1 on bad arguments. */
int st_set_defer_cache(int dtype, unsigned int size_class, unsigned int mask);

/* The size class st_set_defer_ntload indexes for an nrows x ncols block
 * (dtype 0 = f32, 1 = f64), or -1 on a bad dtype. */
int st_defer_ntload_class(unsigned int nrows, unsigned int ncols, int dtype);

/* Cache policy of the every-round flat launch (the vector path): bit 0 turns
 * the matrix loads' policy over (cached <-> non-temporal), bit 1 the
 * stores', 0 = the form's own, per block size class (st_every_cache_class:
 * 0 below 384 MiB, 1 below 640 MiB, 2 below 2 GiB - the cached form - and
 * 3 from 2 GiB - the non-temporal form).  The library's defaults are
 * measured; this overrides one for the process, for
 * tuning tools.  Results do not depend on it.  Returns the previous policy,
 * or -1 on bad arguments. */
int st_set_every_cache(unsigned int size_class, unsigned int policy);

/* Workgroups per CU of the every-round flat launch per size class (the
 * classes of st_set_every_cache; 0 = uncapped, else 2..32), held by dynamic
 * LDS the kernel does not use.  For tuning tools; results do not depend on
 * it.  Returns the previous value, or -1 on bad arguments. */
int st_set_every_caps(unsigned int size_class, unsigned int wg_per_cu);

/* Piece order of the every-round flat launch per size class (the classes of
 * st_set_every_cache): 0 = the library's measured table, 1 = row-major,
 * t > 1 = tiles of t row groups per piece.  For tuning tools; results do not
 * depend on it.  Returns the previous value, or -1 on bad arguments. */
int st_set_every_tile(unsigned int size_class, unsigned int tile);

/* Launch shape of the matrix-free round (k_mfree) for every block of
 * >= 2 x 256 row groups: 0 = the library's measured table, 1 / 2 = cached
 * loads, 2 / 4 rows per group, 3 = non-temporal loads, 4 rows.  For tuning
 * tools; results do not depend on it.  Returns the previous value, or -1
 * on bad arguments. */
int st_set_mfree_shape(unsigned int shape);

/* The size class st_set_every_cache indexes for an nrows x ncols block
 * (dtype 0 = f32, 1 = f64), or -1 on a bad dtype. */
int st_every_cache_class(unsigned int nrows, unsigned int ncols, int dtype);

#ifdef __cplusplus
} /* extern "C" */
#endif

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#endif /* EIGEN_VALUE_AMD_ST_TUNING_H */
