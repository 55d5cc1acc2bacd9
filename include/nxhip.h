/*
 * nxhip.h -- C ABI of the MI355X-native assemble + solve path for the hydraulic
 * network saddle-point system of networks_fenicsx.
 *
 * The reference has no C/FFI boundary of its own: its hot path sits behind the
 * Python classes HydraulicNetworkAssembler and Solver, which hand petsc4py
 * Mat/Vec/KSP objects to DOLFINx C++ and PETSc/MUMPS. Each entry point below
 * names the reference interface it replaces (file:line under
 * /root/reference/src/networks_fenicsx/). The Python binding is
 * networks_fenicsx_amd/_lib.py (ctypes); INTEGRATION.md shows the stub a
 * maintainer would add on the reference side.
 *
 * Conventions
 *   - every function returns NX_OK (0) or a negative NX_ERR_* code; the message
 *     of the last failure on the calling thread is nx_last_error();
 *   - host arrays are caller-owned and copied in/out; device buffers are owned by
 *     the opaque handle and released by nx_destroy;
 *   - calls on one handle must be serialised by the caller (the Python layer holds
 *     the GIL); all work is issued on the handle's own HIP stream.
 *
 * Device layout (per rank): every local graph edge owns 2N+1 consecutive DoFs,
 * interleaved [q_0, p_0, q_1, p_1, ..., p_{N-1}, q_N] (P1 flux vertices and DG0
 * pressure cells, source -> target), then one multiplier per owned bifurcation.
 * Columns >= n_own are ghosts (multipliers or flux end values owned by another
 * rank). The pressure rows are negated so the assembled matrix is symmetric
 * (the solution is unchanged); MINRES requires symmetry.
 */
#ifndef NXHIP_H
#define NXHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NX_OK 0
#define NX_ERR_ARG -1     /* invalid argument / shape */
#define NX_ERR_HIP -2     /* HIP runtime failure */
#define NX_ERR_RCCL -3    /* RCCL failure */
#define NX_ERR_STATE -4   /* call out of order (e.g. solve before assemble) */
#define NX_ERR_NOCONV -5  /* MINRES did not reach the tolerance in maxit */

#define NX_UNIQUE_ID_BYTES 128

typedef struct nx_network nx_network_t;
typedef struct nx_group nx_group_t;

/* Library/ABI version (major*10000 + minor*100 + patch). */
int nx_version(void);

/* Message of the last failure on this thread ("" if none). */
const char* nx_last_error(void);

/* Number of visible HIP devices. */
int nx_device_count(int32_t* count);

/*
 * Create a network handle on `device` and build the CSR sparsity pattern on it.
 * Replaces Solver.__init__'s fem.petsc.create_matrix / create_vector
 * (solver.py:43-49) and the DoF layout of HydraulicNetworkAssembler.__init__
 * (assembly.py:121-162).
 *
 *   N          cells per edge (>= 1)
 *   n_edges    local edges E
 *   edge_x     E*6 doubles: source xyz, target xyz (gdim < 3 padded with 0)
 *   edge_lm    E*2 int32: column of the multiplier at the source / target end,
 *              -1 when that end is not a bifurcation
 *   n_lm       owned multiplier rows B
 *   lm_rowptr  B+1 int32 CSR offsets of the multiplier rows
 *   lm_col     int32 columns (sorted ascending per row): flux end DoFs
 *   lm_val     double values (+1 at an in-edge end q_N, -1 at an out-edge start q_0;
 *              assembly.py:271-277)
 *   n_ghost    ghost columns appended after the n_own = E*(2N+1)+B owned ones
 */
int nx_create(int32_t device, int32_t N, int64_t n_edges, const double* edge_x,
              const int32_t* edge_lm, int64_t n_lm, const int32_t* lm_rowptr,
              const int32_t* lm_col, const double* lm_val, int64_t n_ghost,
              nx_network_t** out);

/*
 * General element degrees: HydraulicNetworkAssembler(mesh, flux_degree=k,
 * pressure_degree=m) (assembly.py:121-146) -- P_k equispaced flux per edge, DG0 (m = 0)
 * or continuous P_m pressure. No tree preconditioner (plain MINRES). The host
 * (networks_fenicsx_amd/layout_fe.py) numbers the DoFs, gives the sorted CSR pattern and
 * lists, for every nonzero and every rhs row, its terms in summation order; the device
 * evaluates them on every nx_assemble (k_assemble_fe: one thread per nonzero / row):
 *
 *   term (idx, ent) = table_val[ent] x factor, factor by table_kind[ent]:
 *     0 constant 1 | 1 R_e h_c (mass; idx = cell e*N + c) | 2 f h_c (source; idx = cell)
 *     | 3 edge_bc[idx] (boundary rhs; idx = 2e + end)
 *   h_c is the cell length from edge_x, computed like the reference mesh generator.
 *
 *   n_rows, rowptr (n_rows+1), col   the symmetric system's CSR pattern (sorted rows)
 *   n_ghost                          several ranks: columns n_rows.. are ghosts
 *                                    (layout_fe.build_fe_rank_layout / build_fe_partition;
 *                                    nx_comm_init then gives the halo plan, as for
 *                                    nx_create); 0 on one rank. n_edges may then count
 *                                    ghost edges too (coefficients, no rows)
 *   n_table, table_kind, table_val   the term table (reference element tensors, signs)
 *   a_ptr (nnz+1), a_idx, a_ent      the terms of every nonzero
 *   b_ptr (n_rows+1), b_idx, b_ent   the terms of every rhs row
 * nx_set_coefficients, nx_assemble, nx_solve and the getters work as for nx_create.
 */
int nx_create_fe(int32_t device, int32_t N, int64_t n_edges, const double* edge_x,
                 int64_t n_rows, const int32_t* rowptr, const int32_t* col, int64_t n_ghost,
                 int32_t n_table, const int32_t* table_kind, const double* table_val, const int32_t* a_ptr,
                 const int32_t* a_idx, const int32_t* a_ent, const int32_t* b_ptr,
                 const int32_t* b_idx, const int32_t* b_ent, nx_network_t** out);

/*
 * The flux degree k when nx_create_fe's tables are exactly a (k, 0) layout's
 * (layout_fe.build_fe_layout with m = 0: every entry's and every rhs row's term list equals
 * the closed form fe_s_terms gives without the tables), else 0. Exported so the host (and
 * the CPU tests) can probe the closed form without a device. Replaces nothing in the
 * reference: its forms are compiled per degree by FFCx (assembly.py:121-146).
 */
int nx_fe_struct_degree(int32_t N, int64_t n_edges, int64_t n_rows, const int32_t* rowptr,
                        const int32_t* col, int32_t n_table, const int32_t* a_ptr,
                        const int32_t* a_idx, const int32_t* a_ent, const int32_t* b_ptr,
                        const int32_t* b_idx, const int32_t* b_ent, int32_t* k_out);

/*
 * The edge templates of a general-degree handle (nx_create_fe builds them when every edge's
 * rows match one of a few shapes): *n_shapes = their number, 0 when the handle kept the
 * gather tables; *rows_per_edge = the rows of one edge. The assembly (k_fe_tasm) and the
 * direct solves' true residual (k_fe_tres) then read no gather tables and no CSR.
 */
int nx_fe_templates(nx_network_t* h, int32_t* n_shapes, int32_t* rows_per_edge);

/* Release every device buffer, graph and communicator of the handle. */
int nx_destroy(nx_network_t* h);

/* Local sizes: owned rows, columns (owned + ghosts), nonzeros. */
int nx_dims(nx_network_t* h, int64_t* n_rows, int64_t* n_cols, int64_t* nnz);

/*
 * Coefficients of the forms (HydraulicNetworkAssembler.compute_forms,
 * assembly.py:165-262), uploaded once and kept resident in HBM:
 *   edge_R   E doubles (per-edge resistance) or NULL to use R_const everywhere
 *   f        constant source term of the pressure equation
 *   edge_bc  E*2 doubles: rhs contribution at q_0 and q_N of each edge
 *            (-p_bc(source) at an inlet root, +p_bc(target) at an outlet leaf,
 *            0 elsewhere; assembly.py:258-260)
 */
int nx_set_coefficients(nx_network_t* h, const double* edge_R, double R_const, double f,
                        const double* edge_bc);

/*
 * Spatially varying source of the mass-conservation equation (the `f` of compute_forms,
 * assembly.py:201-202, 262, given as one value per local edge): edge_f[E] replaces the
 * constant f of nx_set_coefficients in the pressure rhs (f_e h per cell, times the pressure
 * basis integrals for general degrees); NULL returns to the constant.
 */
int nx_set_source(nx_network_t* h, const double* edge_f);

/*
 * Assemble matrix values and/or rhs on the device into the resident CSR.
 * Replaces HydraulicNetworkAssembler.assemble (assembly.py:329-368) and
 * Solver.assemble (solver.py:90-101). Asynchronous on the handle's stream.
 */
int nx_assemble(nx_network_t* h, int32_t lhs, int32_t rhs);

/*
 * Solve on the device; replaces the KSP solve of Solver.solve (solver.py:107-135; default
 * there: preonly + LU/MUMPS). MINRES (Paige-Saunders) by default, or the direct tree solve
 * where nx_set_solver asked for it and it is exact (then iters = 1, or 2 after one
 * refinement step, and relres is the true residual ||b - A x|| / ||b||).
 *   rtol         stop when the MINRES residual estimate ||r_k|| / ||b|| <= rtol
 *   maxit        iteration cap
 *   check_every  iterations per host convergence check (graph chunk), >= 2, even
 *   iters/relres/converged  outputs (host)
 * Returns NX_OK also when not converged; `converged` tells. The solution stays on
 * the device (nx_get_solution copies it out).
 */
int nx_solve(nx_network_t* h, double rtol, int32_t maxit, int32_t check_every,
             int32_t* iters, double* relres, int32_t* converged);

/*
 * Tree Schur-complement preconditioner for MINRES: by default the exact one,
 * P = blockdiag(M, G^T M^{-1} G) with M the consistent flux mass (3 iterations), or with the
 * lumped mass D (nx_set_pc_exact; networks_fenicsx_amd/precond.py derives both and builds
 * these arrays). There is no reference counterpart: the reference factorises with MUMPS
 * (solver.py:58-65); this makes the iterative replacement converge in 3 iterations.
 * enable = 0 switches back to unpreconditioned MINRES. Chains (one per local edge, in job
 * order): edge slot, flip (chain runs target -> source), top / bottom junction slot (-1 =
 * ground). Junction slots (one per owned multiplier, level order per job): multiplier row,
 * chain to the parent, parent slot, CSR of chains hanging below (dc_lo: bottom slot of each
 * entry, slot_plam: the parent's multiplier row -- both derivable, passed to save the
 * kernels a dependent load). Jobs (one workgroup each):
 * chain ranges and level ranges; lvl_slot_off / top_lvl_off: slot offsets per level (root
 * level first) of the lower jobs / of the single top workgroup. Requires N <= 1024.
 * With several ranks the slots also cover the ghost junctions at the ends of local edges
 * (slot_lam = their ghost column) and nx_set_coarse must follow.
 */
int nx_set_preconditioner(nx_network_t* h, int32_t enable, int64_t n_chains,
                          const int32_t* chain_edge, const int32_t* chain_flip,
                          const int32_t* chain_up, const int32_t* chain_lo, int64_t n_slots,
                          const int32_t* slot_lam, const int32_t* slot_pchain,
                          const int32_t* slot_parent, const int32_t* slot_dc_off,
                          const int32_t* slot_dc, const int32_t* dc_lo, const int32_t* slot_plam,
                          int32_t n_jobs, const int32_t* job_chain_off,
                          const int32_t* job_lvl_off, int32_t n_lvl, const int32_t* lvl_slot_off,
                          int32_t n_top_lvl, const int32_t* top_lvl_off);

/*
 * Dense top part (single rank): the down kernel computes the top junction values it
 * needs as rows of G (inverse of the top tree Schur matrix, built once per solve) times
 * the top inputs, which removes the one-workgroup top kernel from every iteration.
 *   job_tslot_off/job_tslot  top slots each job updates and writes (round-robin)
 *   job_need_off/job_need    top slots whose values each job reads (<= 64 per job)
 *   top_uoff[n_top+1]        the top inputs a_s = sum of u[top_uoff[s] .. top_uoff[s+1]),
 *                            posted by the up kernel at fixed places: slot_uy (y' of a top
 *                            slot), chain_uit / chain_uib (I_top / I_bot of a chain, -1 =
 *                            none), job_root_u (kappa J_root + I_top of the root's parent
 *                            chain, kappa = dc entry job_root_dc) -- precond.py
 * Ignored (kept off) with several ranks or when the LDS kernels are not in use;
 * NXHIP_PC_DENSE=0 disables it. Call after nx_set_preconditioner.
 */
int nx_set_pc_dense(nx_network_t* h, int32_t enable, int32_t n_jobs, const int32_t* job_tslot_off,
                    const int32_t* job_tslot, const int32_t* job_need_off,
                    const int32_t* job_need, const int32_t* top_uoff, const int32_t* slot_uy,
                    const int32_t* chain_uit, const int32_t* chain_uib,
                    const int32_t* job_root_u, const int32_t* job_root_dc);

/*
 * Flux mass of the preconditioner: 1 (default) = the consistent P1 mass M, i.e. the exact
 * Schur complement P = blockdiag(M, G^T M^{-1} G) -- P^{-1} A has three distinct eigenvalues
 * and MINRES converges in 3 iterations; 0 = the lumped mass D (O(30) iterations). The
 * junction elimination is the same for both (precond.py, "Exact variant"); only the chain
 * outputs differ. NXHIP_PC_EXACT=0 makes 0 the default. Call after nx_set_preconditioner.
 */
int nx_set_pc_exact(nx_network_t* h, int32_t enable);
int nx_get_pc_exact(nx_network_t* h, int32_t* enabled);

/*
 * Sweep kernels of the preconditioner / direct solve: nx_get_pc_kernels reports whether the
 * uploaded decomposition runs the LDS kernels (1) or the global-memory ones (0, a job over
 * the LDS caps); nx_set_pc_kernels(h, 1) makes the next nx_set_preconditioner take the
 * global-memory kernels even where LDS fits. Several ranks must agree (their exchange
 * schedules differ): the host reduces the ranks' choice (MIN) and re-uploads -- the
 * reference's MPI-collective setup of the solver (solver.py:32-73) in one flag.
 */
int nx_set_pc_kernels(nx_network_t* h, int32_t global);
int nx_get_pc_kernels(nx_network_t* h, int32_t* lds);

/*
 * Which solve nx_solve runs. solver = 0 (default): MINRES. solver = 1: the direct solve
 * the reference's default options ask for (ksp_type=preonly + pc_type=lu + MUMPS,
 * solver.py:58-65), specialised to the network: a block LU of [[M, K], [K^T, 0]] whose
 * Schur complement K^T M^{-1} K is inverted by the tree preconditioner's sweeps --
 *   y = M^{-1} b_q,  x_s = S^{-1} (K^T y - b_s),  x_q = M^{-1} (b_q - K x_s)
 * -- one HIP graph, followed by the true residual ||b - A x|| / ||b|| (one CSR SpMV),
 * which is what nx_solve reports (iters = 1). It runs when it is exact: one rank, the
 * consistent-mass preconditioner (nx_set_pc_exact 1) and tree_exact != 0 (the host
 * decomposition grounded no cycle-closing chain; precond.py TreePreconditioner.tree_exact).
 * Otherwise, or if the residual misses rtol, nx_solve runs MINRES. nx_get_solver returns
 * the requested solver and what the last nx_solve ran (0 MINRES, 1 direct).
 */
int nx_set_solver(nx_network_t* h, int32_t solver, int32_t tree_exact);
int nx_get_solver(nx_network_t* h, int32_t* requested, int32_t* last_run);
/*
 * Graphs with cycles (one rank): the direct solve stays exact, as MUMPS' LU is on any graph
 * (solver.py:58-65; the reference's own cyclic graph, tests/test_edge_info.py:8-35). The
 * decomposition grounds one end of each of the n cycle-closing chains; rows[2i], rows[2i+1]
 * = the flux end row and the multiplier row whose coupling that drops (precond.py
 * TreePreconditioner.cyc_rows). The tree solve inverts A without those n symmetric +-1
 * pairs; nx_solve adds them back with a rank-2n Woodbury correction built once per assembled
 * matrix (2n tree solves of unit vectors, a (2n)^2 capacitance matrix), then checks the true
 * residual with the CSR. n <= 128 (else the solve runs MINRES); n = 0 clears it. Set after
 * every nx_set_preconditioner (which clears it). Replaces nothing one-to-one: MUMPS'
 * factorisation (solver.py:58-65) covers cycles implicitly.
 */
int nx_set_cycles(nx_network_t* h, int32_t n, const int32_t* rows);
/* The same correction with several ranks (RCCL ranks or an in-process group): every rank
 * calls it after nx_set_preconditioner with the cycle chains of ALL ranks in one global
 * order (K pairs, K <= 128; the host control plane gathers them). own[2K]: per column of U
 * (pair k's flux end at 2k, its multiplier at 2k + 1) this rank's row, or -1 where another
 * rank owns it; qloc[K] / lcol[K]: for the pairs whose chain is this rank's, the flux end row
 * and the multiplier's column in this rank's numbering (a ghost column when another rank
 * owns the multiplier row), else -1. Z = A_g^{-1} U is built by 2K team tree solves, U^T Z
 * and the couplings are summed over the ranks (one all-reduce), every rank inverts the same
 * capacitance matrix; per solve U^T x is summed (one all-reduce of 2K), x -= Z Cinv U^T x on
 * every rank's rows, and the true residual comes from the CSR after a halo of x. The cycle
 * count is part of the ranks' schedule signature. K = 0 clears it. Replaces MUMPS'
 * distributed factorisation of a cyclic graph (solver.py:58-65, mesh.py:341-348). */
int nx_set_cycles_team(nx_network_t* h, int32_t K, const int32_t* own, const int32_t* qloc,
                       const int32_t* lcol);

/*
 * General flux degree k >= 2 with DG0 pressure (assembly.py:121-146, flux_degree=k), one
 * rank: the direct solve through the condensed system. The DG0 divergence touches a cell's
 * two vertex fluxes only, so the k-1 interior fluxes per cell are condensed out per cell;
 * what remains has the P1/DG0 structure with the cell mass R h [[a, b], [b, a]]
 * (element.condensed_flux_mass: k = 2: a = 1/8, b = -1/24). An auxiliary P1/DG0 handle of
 * the same graph (nx_create + its tree preconditioner, nx_set_solver 1) inverts it.
 *
 * nx_set_cell_mass(aux, ratio, mo_div): the auxiliary handle's flux mass is the condensed
 *   one, ratio = a / b (T = tridiag(1, 2 ratio, 1), ratio at both ends; P1: 2) and mo_div =
 *   (a + b) / b (P1: 3). The handle is internal from then on: its own CSR is no longer the
 *   system its sweeps invert (it checks no residual; nx_solve on it runs MINRES).
 * nx_fe_set_direct(h, aux, k, n_lm, ...): attaches aux to the (k, 0) handle h (nx_create_fe):
 *   slot[e] = aux edge of h's edge e; v_fe / v_aux (E (N+1)) the vertex-flux rows, edge-major;
 *   i_fe (E N (k-1)) the interior-flux rows, cell-major; p_fe / p_aux (E N) pressure rows;
 *   l_fe / l_aux (n_lm) multiplier rows; cst = C (2 x (k-1)) | K ((k-1) x 2) | M_ii^{-1}
 *   ((k-1)^2), row-major; ab = a + b. aux = NULL detaches. With nx_set_solver(h, 1, 1),
 *   nx_solve condenses, solves on aux, expands, checks h's true residual and refines up to
 *   twice (iters = passes), MINRES when that still misses rtol. layout_fe.build_fe_aux_maps
 *   builds the maps. Replaces MUMPS' LU of the (k, 0) system (solver.py:58-65).
 *   Several ranks: h (n_ghost > 0) and aux (the rank's P1/DG0 handle with its halo, cut rows
 *   and preconditioner) each joined to the ranks' communicator; the aux solve is the ranks'
 *   direct tree solve, h's residual takes the halo of x and one all-reduce.
 */
int nx_set_cell_mass(nx_network_t* aux, double ratio, double mo_div);
int nx_fe_set_direct(nx_network_t* h, nx_network_t* aux, int32_t k, int64_t n_lm,
                     const int32_t* slot, const int32_t* v_fe, const int32_t* v_aux,
                     const int32_t* i_fe, const int32_t* p_fe, const int32_t* p_aux,
                     const int32_t* l_fe, const int32_t* l_aux, const double* cst, double ab);

/*
 * Continuous pressure (pressure_degree m >= 1, flux_degree k > m; assembly.py:121-146), one
 * rank, a forest: the direct solve by condensation onto the graph nodes, replacing MUMPS'
 * LU (solver.py:58-65) for these pairs. Each edge's own unknowns (its kN+1 flux nodes and
 * mN-1 interior pressure nodes) are eliminated onto its border: the pressure at its two end
 * nodes (shared with the other edges there) and the multipliers of the bifurcations at its
 * ends. Per cell the interior nodes condense onto the vertices by exact reference blocks
 * scaled by s = R h (layout: element.condensed_cell_blocks); per edge the vertices (q, p)
 * are eliminated along it (one thread per edge); the border system over the graph nodes
 * (negative definite, 2 unknowns per node) is eliminated leaf to root by one workgroup;
 * then every edge back-substitutes. The true residual comes from the CSR, with up to two
 * refinement passes; nx_get_direct_path reports 4.
 *   nI = (k-1)+(m-1); cst = Kh (16) | Ch (4 nI) | Eh (4 nI) | Fh (nI nI); tI[nI] (+1 flux,
 *   -1 pressure interior node); n_nodes border nodes, nrow[2n] (pressure row, multiplier row
 *   or -1); eb[4E] (source node, target node, the q_0 - lam_source and q_N - lam_target
 *   couplings: 0 or +-1); the node forest: n_lev levels (lev_off, order), every node's
 *   (edge, end) incidences (inc_off, inc), parent[3n] (parent node, edge, this node's end of
 *   it; -1 at a root), children (child_off, child), nown[n] (the edge that writes the node's
 *   rows). k = 0 detaches it. Built by layout_fe.build_cp_tables.
 */
int nx_fe_set_cp(nx_network_t* h, int32_t k, int32_t m, int32_t nI, const double* cst,
                 const int32_t* tI, int64_t n_nodes, const int32_t* nrow, const int32_t* eb,
                 int32_t n_lev, const int32_t* lev_off, const int32_t* order,
                 const int32_t* inc_off, const int32_t* inc, const int32_t* parent,
                 const int32_t* child_off, const int32_t* child, const int32_t* nown);

/*
 * Several ranks, continuous pressure (called before nx_fe_set_cp; layout_fe.
 * build_cp_rank_tables): this rank runs the edge kernels on its n_own_edges edges (gid: each
 * one's global edge), every rank's border blocks and the node rows' rhs are summed over the
 * ranks (one all-reduce per pass), every rank solves the node forest, and each writes the
 * node rows it owns (nrowx, 2 per node: local rows or -1). nx_fe_set_cp's eb / nown then
 * list this rank's edges (nown: -1 where another rank writes the node), its nrow the node
 * rhs slots (2n, 2n + 1 or -1), its incidence and parents global edges. Replaces the
 * distributed MUMPS LU (solver.py:58-65) for these pairs.
 */
int nx_fe_cp_ranks(nx_network_t* h, int64_t n_own_edges, int64_t n_edges_global,
                   const int32_t* gid, int64_t n_nodes, const int32_t* nrowx);

/*
 * Process-wide solve mode. 1 (default): with the preconditioner a solve is ONE HIP graph
 * launch -- start application, per-solve coefficients and the first iterations (also with
 * several ranks, RCCL or group, when beta^2 travels point-to-point) -- whose last k_mr_a
 * publishes the MINRES state to host-coherent memory; nx_solve returns once it is
 * published (the final solution update may still run: every host read of device data
 * synchronises the stream). 0: eager prologue, chunked iteration graphs, a stream
 * synchronisation per chunk (the path profiling always uses). NXHIP_LEAN=0 sets 0.
 */
int nx_set_lean(int32_t enable);

/*
 * Coarse step of the preconditioner on a partitioned problem (precond.py derives it): the
 * coarse junctions (interface junctions + the junctions on paths between them inside a
 * rank) form a forest that every rank solves redundantly from one all-reduce of
 * [D | J | G] (3 n_coarse doubles) per application, which keeps P^{-1} exact, i.e. the
 * iteration count independent of the number of ranks.
 *   slot_cidx[n_slots]        coarse index of every slot, -1 (coarse slots: top part)
 *   cc_chain/cc_top/cc_bot    local chains joining two coarse junctions: chain, coarse
 *                             index of its top / bottom end (the bottom is the child)
 *   c_parent[n_coarse], c_child_off/c_child (CSR), c_lvl_off[n_clvl+1]: the global
 *                             forest in level order (root level first)
 * n_coarse = 0 disables the step. Call after nx_set_preconditioner.
 */
int nx_set_coarse(nx_network_t* h, int32_t n_coarse, const int32_t* slot_cidx, int32_t n_cc,
                  const int32_t* cc_chain, const int32_t* cc_top, const int32_t* cc_bot,
                  const int32_t* c_parent, const int32_t* c_child_off, const int32_t* c_child,
                  int32_t n_clvl, const int32_t* c_lvl_off);

/* 1 if the last nx_solve replayed its iterations as HIP graphs (also with RCCL, unless
 * the capture failed or NXHIP_RCCL_GRAPH=0), 0 if it launched them one by one. */
int nx_get_graph_mode(nx_network_t* h, int32_t* graph);

/* Copy the owned part of the solution / rhs to the host (n_rows doubles). */
int nx_get_solution(nx_network_t* h, double* x);
int nx_get_rhs(nx_network_t* h, double* b);

/* The solution in the reference's function order -- what Solver.solve assigns into
 * [flux_color_0 .. flux_color_{M-1}, pressure, global_flux] (solver.py:120-134,
 * dolfinx.fem.petsc.assign). nx_set_output_map uploads once the permutation `rows`
 * (n_rows entries, a permutation of the owned rows: output position -> device row);
 * nx_get_solution_blocks gathers x into that order on the device and copies it to `out`
 * (n_rows doubles; pinned memory from nx_host_alloc makes the copy one DMA at PCIe
 * speed). Synchronous: `out` is complete when it returns. */
int nx_set_output_map(nx_network_t* h, int64_t n, const int32_t* rows);
int nx_get_solution_blocks(nx_network_t* h, double* out);

/* Deferred form of nx_get_solution_blocks (what Solver.solve returns by default):
 * nx_snapshot_solution gathers x into the function order into the handle's device
 * snapshot `slot` (0 <= slot < 64, allocated on first use) on the handle's stream and
 * returns without waiting -- later solves do not disturb it; nx_fetch_snapshot copies a
 * slot to `out` (n_rows doubles) on a separate copy stream once the gather has run and
 * waits for that copy only. The caller owns the slot bookkeeping (a slot is rewritten by
 * the next nx_snapshot_solution into it). Replaces the same assign as above
 * (solver.py:120-134): the functions' host arrays are filled when first read. */
int nx_snapshot_solution(nx_network_t* h, int32_t slot);
int nx_fetch_snapshot(nx_network_t* h, int32_t slot, double* out);

/* Page-locked host memory for nx_get_solution_blocks (hipHostMalloc / hipHostFree). */
int nx_host_alloc(int64_t bytes, void** out);
int nx_host_free(void* p);

/* Owned part of an internal vector (n_rows doubles): 0 = solution, 1 = rhs,
 * 2 = the latest preconditioned residual z = P^{-1} r (with the preconditioner). */
int nx_get_vector(nx_network_t* h, int32_t which, double* out);

/* Copy the assembled CSR (n_rows+1, nnz, nnz) to the host -- parity tests. */
int nx_get_csr(nx_network_t* h, int32_t* rowptr, int32_t* col, double* val);

/* y = A x for host vectors (x has n_cols entries incl. ghosts) -- tests. */
int nx_spmv_host(nx_network_t* h, const double* x, double* y);

/* True residual ||b - A x|| / ||b|| of the current device solution. */
int nx_true_residual(nx_network_t* h, double* relres);

/* Wait for all work queued on the handle's stream. */
int nx_sync(nx_network_t* h);

/*
 * Kernel timing with HIP events on the handle's stream.
 *   nx_set_profiling(h, 1) brackets every SpMV launch inside nx_solve with an
 *   event pair; nx_get_profile returns the summed SpMV time (ms), the number of
 *   timed SpMV launches, and the summed assembly kernel time (ms).
 *   nx_bench_spmv times `reps` back-to-back plain SpMV launches (ms per launch).
 */
int nx_set_profiling(nx_network_t* h, int32_t enable);
int nx_get_profile(nx_network_t* h, double* spmv_ms, int64_t* spmv_count, double* asm_ms,
                   int64_t* asm_count);
/* Direct solve (nx_set_solver 1, profiling on): summed kernel times (ms) of the up, top and
 * down sweeps (mode kModeDirect) and of the residual SpMV, over `count` direct solves, each
 * from events bound to the kernel's own dispatch (no graph while profiling). */
int nx_get_profile_direct(nx_network_t* h, double* ms4, int64_t* count);
/* How the direct solve checks its residual: *fused = 1 when the down sweep forms r = b - A x
 * itself (one rank, LDS kernels; the 4th time of nx_get_profile_direct is then the publish
 * kernel k_dir_publish_fr, which also forms the *n_left multiplier rows of the top part from
 * the CSR), 0 when a separate CSR SpMV (k_residual_ck) does. */
int nx_get_direct_info(nx_network_t* h, int32_t* fused, int32_t* n_left);
/* What the last direct solve ran: *path = 1 for the fused step k_dir_step (one rank, the
 * deferred assembly + the whole tree solve + the residual check + the published state in
 * one launch; under profiling its time is the 1st of nx_get_profile_direct, the others 0),
 * 0 for the separate launches (assembly, up sweep, down sweep, publish). Replaces nothing
 * in the reference (PETSc's KSPSolve is one call: solver.py:127). */
int nx_get_direct_path(nx_network_t* h, int32_t* path);
/* Whether the last fused or exchange step (path 1 or 3) ran phase 2 by superposition
 * (*sup = 1: the instantiation k_dir_step / k_dir_xr <W, CPL, true>, NXHIP_DIR_SUP; 0: the
 * plain phase 2). Replaces nothing in the reference (its profiling names). */
int nx_get_direct_sup(nx_network_t* h, int32_t* sup);
/* (path 2: the (k, 0) condensed route of nx_fe_set_direct; path 4: the continuous-pressure
 * node-condensed route of nx_fe_set_cp; path 3: several ranks, the
 * exchange step k_dir_xr / k_dir_xg, one launch per rank.)
 * Test hook: the number of s_sleep-paced polls a k_dir_step workgroup spends waiting for the
 * top part's values before it gives up (default 2^20). 0 makes every waiting workgroup give
 * up at once, which forces the fallback a non-co-resident launch takes: the host resets the
 * hand-off counters and the device's published-state count and runs the separate launches
 * on this handle from then on (until the next nx_set_preconditioner). Replaces nothing in
 * the reference. */
int nx_debug_set_wait_polls(nx_network_t* h, uint32_t polls);
/* Rehearsal hook: the exchange step (k_dir_xr) of group member h ALONE, reps timed launches
 * (*ms: average kernel time, HIP events on the dispatch), its two exchanges emulated from
 * the sums the group's previous graph-path direct solve left -- the per-rank time of a
 * multi-GPU run measured on one GPU (whose ranks cannot all be resident in one launch).
 * h's solution is then the rank's share of the answer. Replaces nothing in the reference. */
int nx_debug_xr_rehearse(nx_network_t* h, double rtol, int32_t reps, double* ms);

/* Debug / tests: the RCCL ranks' shape of the exchange step on one GPU -- every rank of the
 * group launches its own k_dir_xr on a stream of its own (concurrent launches meeting only
 * through the mailboxes, the exchange width the handle's rank count), the ranks' assembly
 * pending. *relres = the published residual (every rank's equal). */
int nx_debug_xr_separate(nx_group_t* g, double rtol, double* relres);
/* A rank that gives up an exchange raises an abort word in every rank's mailbox, so the
 * other ranks' exchanges fail at once; the ranks then agree, through one max-all-reduce of
 * four doubles, on who finished which step, so every rank leaves the exchange step at the
 * same point and no collective of the graph path is ever paired across steps (the rank that
 * gave up exchange 2 of a step the others finished keeps its final x and takes their
 * published residual). Test hook: the poll bound of this rank's exchange `which` (0: the
 * coarse partials, 1: the residual) in its next steps; 0 makes it give up at once, after
 * its own slots and flags are written. Replaces nothing in the reference. */
int nx_debug_xr_polls(nx_network_t* h, int32_t which, uint32_t polls);
/* out[4] = [the exchange step is off for good (agreed), the last launch's give-up reasons
 * (bits: 1 exchange 1, 2 exchange 2, 4 another rank's abort seen, 8 a slot with another
 * launch's tag, 16 a local wait), agreements this rank took part in, the last launch's tag]. */
int nx_get_xr_status(nx_network_t* h, int32_t* out);
int nx_reset_profile(nx_network_t* h);
int nx_bench_spmv(nx_network_t* h, int32_t reps, double* ms_per_spmv);
/* The same SpMV rotating over private copies of the CSR and vectors (> 512 MiB in total,
 * twice the Infinity Cache) so every launch streams from HBM ("cold"). */
int nx_bench_spmv_cold(nx_network_t* h, int32_t reps, int32_t* copies, double* ms_per_spmv);

/*
 * Multi-GPU (one process per GPU). Rank 0 creates the RCCL unique id, the
 * host control plane (torch.distributed) broadcasts it, every rank calls
 * nx_comm_init with its halo plan. Replaces the MPI ghost updates
 * (assembly.py:363-367, solver.py:128-132) and MUMPS' internal communication.
 *   n_peers                 neighbouring ranks
 *   peer_rank[n_peers]
 *   send_off[n_peers+1], send_idx[...]   owned local rows to send to each peer
 *   recv_off[n_peers+1]     ghost slots [recv_off[p], recv_off[p+1]) filled by peer p
 * nx_set_halo records the plan only; nx_comm_init = nx_set_halo + the RCCL communicator.
 * Both must precede nx_set_preconditioner.
 */
int nx_comm_unique_id(unsigned char* id_out /* NX_UNIQUE_ID_BYTES */);
int nx_set_halo(nx_network_t* h, int32_t nranks, int32_t rank, int32_t n_peers,
                const int32_t* peer_rank, const int32_t* send_off, const int32_t* send_idx,
                const int32_t* recv_off);
int nx_comm_init(nx_network_t* h, int32_t nranks, int32_t rank, const unsigned char* id,
                 int32_t n_peers, const int32_t* peer_rank, const int32_t* send_off,
                 const int32_t* send_idx, const int32_t* recv_off);
/* Tests: nx_comm_init with a host transport in place of RCCL -- several ranks' processes on
 * ONE GPU (RCCL refuses two ranks on one device), collectives through the POSIX shared
 * memory `name` ("/..."; the same on every rank, chosen by rank 0 and broadcast), eager
 * (every collective synchronises the stream; no graph capture). It runs the RCCL ranks' host
 * logic unchanged: the exchange step over IPC-mapped mailboxes, its agreement, the graph
 * path. Not a performance path. Replaces nothing in the reference. */
int nx_comm_init_host(nx_network_t* h, int32_t nranks, int32_t rank, const char* name,
                      int32_t n_peers, const int32_t* peer_rank, const int32_t* send_off,
                      const int32_t* send_idx, const int32_t* recv_off);

/* Several ranks, direct solve: the multiplier rows of the K cut bifurcations (incident
 * edges on several ranks; one global order, the same on every rank) are completed inside
 * the residual's all-reduce of [||r||^2, ||b||^2, r_cut[K]] instead of a halo of x and a
 * second all-reduce -- the MPI ghost update + norm of the reference's solve
 * (solver.py:128-132, assembly.py:363-367) in one collective.
 *   lm_cut[n_lm]        per owned multiplier row (local order): its cut index or -1
 *   gk_off[K+1], gk_row, gk_coef   per cut index owned by another rank: this rank's flux
 *                       end rows at it and their coupling coefficient (+-1)
 * NXHIP_DIR_CUT=0 keeps the halo path. Part of the ranks' schedule signature. */
int nx_set_cut(nx_network_t* h, int32_t K, const int32_t* lm_cut, const int32_t* gk_off,
               const int32_t* gk_row, const double* gk_coef);

/* Several ranks, direct solve in ONE launch per rank (k_dir_xr): the ranks exchange the
 * coarse partials and the residual's partials device-side, through a mailbox in each rank's
 * device memory that every rank writes into (IPC-mapped over xGMI) -- no RCCL call in the
 * step. After nx_comm_init: nx_xch_export writes this rank's mailbox handle
 * (NX_XCH_HANDLE_BYTES); the host control plane all-gathers them in rank order; every
 * rank passes all P to nx_xch_import. The ranks decide together (the schedule comparison)
 * whether every one can run the step; otherwise the graph path (RCCL all-reduces) runs.
 * NXHIP_DIR_XR=0 keeps the graph path. Replaces the MPI reductions of the reference's
 * distributed MUMPS solve (solver.py:127-132); in-process groups link their mailboxes in
 * nx_group_create. */
#define NX_XCH_HANDLE_BYTES 64
int nx_xch_export(nx_network_t* h, unsigned char* handle_out);
int nx_xch_import(nx_network_t* h, const unsigned char* handles);

/* Ranks of the handle's RCCL communicator (ncclCommCount); without one, the rank count of
 * its halo plan (1 for a single-GPU handle). bench.py reports it next to the timing. */
int nx_comm_count(nx_network_t* h, int32_t* nranks);

/*
 * In-process rank group: the ranks of a partitioned problem as handles on ONE device,
 * driven in lock-step from one host thread, with the halo exchange as device copies and
 * the all-reduces as a fixed-order device sum. Same kernels and schedule as the RCCL path,
 * so a multi-rank solve can be checked on a single GPU (RCCL rejects two ranks on one
 * device). Each handle h_r needs nx_set_halo(h_r, nranks, r, ...) first; the group lends
 * the handles one shared stream until nx_group_destroy (which must precede nx_destroy).
 * nx_group_solve = nx_solve over all ranks; fails with NX_ERR_STATE if the ranks' MINRES
 * recurrences ever differ.
 */
int nx_group_create(int32_t nranks, nx_network_t* const* handles, nx_group_t** out);
int nx_group_solve(nx_group_t* g, double rtol, int32_t maxit, int32_t check_every,
                   int32_t* iters, double* relres, int32_t* converged);
int nx_group_destroy(nx_group_t* g);

#ifdef __cplusplus
}
#endif

#endif /* NXHIP_H */
