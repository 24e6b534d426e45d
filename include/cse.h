/*
 * cse.h -- C ABI of the MI355X (gfx950) residual/Jacobian evaluator.
 *
 * "cse" = Ceres Solver Evaluator.  This is the drop-in boundary for the hot
 * path of jwmak/ceres-solver-cuda: the per-residual-block autodiff evaluator
 * behind ProblemCUDA.  Every entry point names the reference interface it
 * replaces (paths relative to the reference checkout).
 *
 * Plain C: no exceptions cross the boundary, no torch/HIP types in the
 * signatures (streams are passed as void*), every buffer is a pointer plus
 * a size.  All functions return 0 on success, a positive status for a
 * numerical failure (a residual block reported failure) and a negative
 * status for a usage or HIP error; cse_last_error() then describes it.
 *
 * Threading: an evaluator is not thread-safe (the reference's
 * RegisteredCUDAEvaluators is not either).  Distinct evaluators may be used
 * from distinct threads.
 */
#ifndef CSE_H_
#define CSE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: cse_parameter_block.manifold (was `reserved`, which had to be 0),
 *    cse_host_register / cse_host_unregister, cse_shard_transfer_bytes,
 *    shard-local state in cse_create_multi.
 * 3: cse_options.jacobian_form.
 * 4: user functor kinds (cse_register_functor, cse_functor_shape),
 *    CSE_LOSS_USER and cse_loss.user, cse_schur_init_gradient.
 * 5: cse_functor_ops.fused_points / camera_gradient (the fused gradient for
 *    user kinds) and camera_gradient_args_size (was reserved[0]). */
#define CSE_ABI_VERSION 5

/* Return codes. */
#define CSE_OK 0
#define CSE_EVALUATION_FAILED 1 /* a functor returned false / non-finite output */
#define CSE_ERR_INVALID -1      /* malformed descriptor or arguments */
#define CSE_ERR_HIP -2          /* HIP runtime error */
#define CSE_ERR_OOM -3          /* device allocation failed */
#define CSE_ERR_UNSUPPORTED -4  /* functor/loss/layout not available */

/* Residual functors pre-instantiated in the library.  The reference
 * compiles user functors header-only into the user's nvcc TU
 * (include/ceres/problem_cuda.h:110-160); across a C ABI the functor is a
 * kind plus per-block constants ("functor data").
 *   kind                                  kR  blocks  data
 *   SNAVELY_2_9_3                          2  9,3     obs_x, obs_y
 *       examples/snavely_reprojection_error.h:54-105
 *   SNAVELY_NO_DISTORTION_2_7_3            2  7,3     obs_x, obs_y
 *       internal/ceres/evaluator_cuda_test.cu.cc:112-150
 *   SNAVELY_QUATERNION_2_10_3              2  10,3    obs_x, obs_y
 *       examples/snavely_reprojection_error.h:112-175
 *   POINT_DISPLACEMENT_3_3                 3  3       x, y, z
 *       internal/ceres/evaluator_cuda_test.cu.cc:84-110
 */
typedef enum cse_functor_kind {
  CSE_FUNCTOR_SNAVELY_2_9_3 = 0,
  CSE_FUNCTOR_SNAVELY_NO_DISTORTION_2_7_3 = 1,
  CSE_FUNCTOR_SNAVELY_QUATERNION_2_10_3 = 2,
  CSE_FUNCTOR_POINT_DISPLACEMENT_3_3 = 3,
  /* The functors of the reference's own known-answer tests, so that those
   * tests run through the library's kernels (general path, trivial loss
   * only).  kind                      kR  blocks      data
   *   TEST_LINEAR_<kR>_<sizes>           see name    kFactor, succeeds
   *       ParameterIgnoringCostFunction, internal/ceres/evaluator_test.cc:58-100,
   *       as r_i = (i+1) + kFactor sum_b sum_j (j+1) x_b[j] (exact at x = 0)
   *   TEST_BILINEAR_1_2_2             1   2,2         a
   *       BinaryScalarCost, autodiff_cost_function_cuda_test.cu.cc:40-51
   *   TEST_TEN_PARAMETER_1_x10        1   1 (x10)     unused
   *       TenParameterCost, autodiff_cost_function_cuda_test.cu.cc:123-139
   *   TEST_PARTIAL_OUTPUT_2_1         2   1           unused
   *       OnlyFillsOneOutputFunctor, autodiff_cost_function_cuda_test.cu.cc:224-230 */
  CSE_FUNCTOR_TEST_LINEAR_3_2_3_4 = 100,
  CSE_FUNCTOR_TEST_LINEAR_3_4_3_2 = 101,
  CSE_FUNCTOR_TEST_LINEAR_2_2_3 = 102,
  CSE_FUNCTOR_TEST_LINEAR_3_2_4 = 103,
  CSE_FUNCTOR_TEST_LINEAR_4_3_4 = 104,
  CSE_FUNCTOR_TEST_BILINEAR_1_2_2 = 110,
  CSE_FUNCTOR_TEST_TEN_PARAMETER_1_x10 = 111,
  CSE_FUNCTOR_TEST_PARTIAL_OUTPUT_2_1 = 112
} cse_functor_kind;

/* LossFunctionCUDA variants, include/ceres/loss_function_cuda.h:62-150. */
typedef enum cse_loss_kind {
  CSE_LOSS_TRIVIAL = 0, /* TrivialLossCUDA (or nullptr, problem_cuda.h:146-160) */
  CSE_LOSS_HUBER = 1,   /* HuberLossCUDA(a) */
  CSE_LOSS_CAUCHY = 2,  /* CauchyLossCUDA(a) */
  /* A user LossFunctionCUDA type (a class with
   *   __host__ __device__ void Evaluate(double s, double rho[3]) const,
   * the contract of loss_function_cuda.h:62-94), compiled into a user functor
   * kind's kernels (cse_functor_ops.loss_kind); the group's object is passed
   * as bytes in cse_loss.user.  Only with such a kind. */
  CSE_LOSS_USER = 3
} cse_loss_kind;

#define CSE_USER_LOSS_BYTES 64

typedef struct cse_loss {
  int32_t kind;   /* cse_loss_kind */
  int32_t scaled; /* 1 = wrapped in ScaledLossCUDA(rho, scale) */
  double a;       /* loss parameter a */
  double scale;   /* ScaledLossCUDA factor */
  /* CSE_LOSS_USER: the loss object's bytes (trivially copyable, at most
   * CSE_USER_LOSS_BYTES), handed to the kernels as they are. */
  double user[CSE_USER_LOSS_BYTES / 8];
} cse_loss;

/* One parameter block of the reduced Program; replaces ParameterBlockCUDA
 * (include/ceres/internal/parameter_block_cuda.h:106-116) as filled by
 * RegisteredCUDAEvaluators::SetupParameterBlocks
 * (internal/ceres/registered_cuda_evaluators.cc:123-198). */
typedef struct cse_parameter_block {
  int32_t size;                 /* ambient size */
  int32_t tangent_size;         /* == size without a manifold */
  int32_t is_constant;          /* held constant: no Jacobian, no gradient */
  int32_t manifold;             /* cse_manifold_kind (ABI 1: `reserved`, 0) */
  int64_t state_offset;         /* into state (active) / constant_state (constant) */
  int64_t delta_offset;         /* into the gradient (active only) */
  int64_t plus_jacobian_offset; /* into plus_jacobians (size x tangent row-major), -1 = none */
} cse_parameter_block;

/* How the evaluator gets a block's plus-Jacobian (Manifold::PlusJacobian).
 *   CSE_MANIFOLD_MATRIX: the size x tangent_size matrix at
 *       plus_jacobian_offset, refreshed by cse_set_plus_jacobians, as the
 *       reference uploads it (registered_cuda_evaluators.cc:139-160);
 *       plus_jacobian_offset -1 = no manifold.
 *   CSE_MANIFOLD_QUATERNION_EUCLIDEAN: ProductManifold<QuaternionManifold,
 *       EuclideanManifold<size - 4>> (Ceres order w, x, y, z first; the
 *       --use_quaternions --use_manifolds camera of examples/bundle_adjuster.cc:
 *       337-345 and evaluator_cuda_test.cu.cc:286): tangent_size = size - 1,
 *       plus_jacobian_offset must be -1.  The kernels build the plus-Jacobian
 *       (QuaternionPlusJacobianImpl, internal/ceres/manifold.cc:62-78, and an
 *       identity block) from the block's current value in registers; the
 *       result equals the dense product with that matrix.  Blocks of this kind
 *       in slot 0 of SNAVELY_QUATERNION_2_10_3 groups keep the affine (fast)
 *       kernels; cse_plus applies QuaternionPlusImpl (manifold.cc:28-59) to
 *       them and x + delta to the Euclidean part. */
typedef enum cse_manifold_kind {
  CSE_MANIFOLD_MATRIX = 0,
  CSE_MANIFOLD_QUATERNION_EUCLIDEAN = 1
} cse_manifold_kind;

/* All residual blocks of one (functor kind, loss) type; replaces one
 * AutoDiffResidualBlockCUDAEvaluator<F, Loss, kR, Ns...> and its residual
 * blocks (include/ceres/internal/autodiff_residual_block_cuda_evaluator.h:62-334,
 * registered per std::type_index in problem_cuda.h:462-468).  The loss is
 * uniform over the group (one loss object per type is what ProblemCUDA
 * users register in practice; groups may be split to vary it). */
typedef struct cse_residual_group {
  int32_t functor_kind;               /* cse_functor_kind */
  int32_t reserved;
  cse_loss loss;
  int64_t num_blocks;
  /* Global residual block index (program order, ResidualBlock::index())
   * of block i; NULL means first_residual_block + i. */
  const int64_t* residual_block_index;
  int64_t first_residual_block;
  /* [num_blocks][num parameter blocks of the kind], program indices. */
  const int32_t* parameter_block_ids;
  /* [num_blocks][data size of the kind] functor constants. */
  const double* functor_data;
} cse_residual_group;

/* The reduced Program plus the Jacobian layout the evaluator writes into:
 * the arguments of RegisteredCUDAEvaluators::Init
 * (internal/ceres/registered_cuda_evaluators.cc:226-280), with int64 offsets
 * (the reference's int32 overflows past ~89M observations). */
typedef struct cse_problem_desc {
  int32_t abi_version; /* CSE_ABI_VERSION */
  int32_t num_groups;
  const cse_residual_group* groups;

  int64_t num_parameter_blocks;
  const cse_parameter_block* parameter_blocks;
  int64_t num_parameters;           /* Program::NumParameters (state size) */
  int64_t num_effective_parameters; /* Program::NumEffectiveParameters */
  int64_t num_constant_parameters;  /* Program::NumConstantParameters */
  const double* constant_state;     /* host, copied once (registered_cuda_evaluators.cc:237-248) */
  int64_t num_plus_jacobian_values;
  const double* plus_jacobians;     /* host; refresh with cse_set_plus_jacobians */

  int64_t num_residual_blocks;
  int64_t num_residuals;
  /* ProgramEvaluatorCUDA::BuildResidualLayout (program_evaluator_cuda.h:159-170). */
  const int64_t* residual_layout;
  /* {BlockJacobianWriter,CompressedRowJacobianWriter}::CreateJacobianPerResidualLayout
   * (block_jacobian_writer.cc:154-160, compressed_row_jacobian_writer.cc:240-300). */
  const int64_t* jacobian_per_residual_layout;
  const int64_t* jacobian_per_residual_offsets;
  int64_t num_jacobian_per_residual_offsets;
  int64_t num_jacobian_values; /* SparseMatrix::num_nonzeros() */
} cse_problem_desc;

typedef struct cse_options {
  int32_t device;               /* HIP device ordinal; -1 = current device */
  int32_t check_finite;         /* reject non-finite r/J (residual_block.cc:110-129) */
  int32_t apply_loss_function;  /* Evaluator::EvaluateOptions::apply_loss_function */
  int32_t force_general_layout; /* never take the affine fast path (testing) */
  int32_t profile;              /* time every evaluate kernel with HIP events */
  int32_t use_stream;           /* 1: run on `stream` as given, even NULL (the null stream) */
  void* stream;                 /* hipStream_t to run on; NULL and use_stream 0 =
                                   an evaluator-owned stream */
  int32_t gradient_mode;        /* how g = J^T r is summed when the residuals and
                                   Jacobian are requested too: 0 (default) = fused
                                   where eligible (slot-1 rows in the evaluation,
                                   slot-0 rows by re-evaluation in slot-0 order),
                                   else 1; 1 = a fixed-order post-pass over the
                                   written Jacobian; 2 = in-kernel FP64 atomics,
                                   as cuda_evaluator_kernel.h:149-160; 3 = fused,
                                   slot-0 contributions written in block order and
                                   summed per block (the round-2 form), else 1.
                                   0, 1 and 3 are bit-deterministic.  With
                                   jacobian_form CSE_JACOBIAN_JET, and for user
                                   kinds, 3 runs as 1. */
  int32_t jacobian_form;        /* cse_jacobian_form: how the SnavelyReprojectionError
                                   Jacobian is differentiated (every other kind always
                                   uses Jet<double, N>, AutoDifferentiate) */
} cse_options;

/* cse_options.jacobian_form.  Both give the Jacobian of the same functor to
 * within the parity bounds; the closed form is faster (fewer FP64 operations,
 * fewer registers). */
typedef enum cse_jacobian_form {
  /* Snavely<2,9,3>: the forward-mode product rule written out once in closed
   * form (SnavelyJacobianByHand); the default. */
  CSE_JACOBIAN_CLOSED_FORM = 0,
  /* Forward-mode dual numbers Jet<double, 12> seeded per parameter, as
   * AutoDiffCostFunction / AutoDifferentiate (autodiff.h:314-381,
   * autodiff_cost_function_cuda.h:55-71). */
  CSE_JACOBIAN_JET = 1
} cse_jacobian_form;

typedef struct cse_evaluator cse_evaluator;

/* Fills *options with the defaults: device -1, check_finite 1,
 * apply_loss_function 1, everything else 0 (an evaluator-owned stream). */
void cse_default_options(cse_options* options);

/* Replaces RegisteredCUDAEvaluators::Init + each
 * AutoDiffResidualBlockCUDAEvaluator::Init (uploads topology, layouts and
 * constants once).  The descriptor's host arrays are copied; they may be
 * freed after the call. */
int cse_create(const cse_problem_desc* desc, const cse_options* options,
               cse_evaluator** out);

/* Replaces RegisteredCUDAEvaluators::Evaluate
 * (include/ceres/internal/registered_cuda_evaluators.h:75-79): host
 * pointers, any output except cost may be NULL, synchronous.  Returns
 * CSE_OK, CSE_EVALUATION_FAILED (Evaluate returning false) or an error. */
int cse_evaluate(cse_evaluator* ev, const double* state, double* cost,
                 double* residuals, double* gradient, double* jacobian_values);

/* Device-resident variant (no host copies; the roofline path): all pointers
 * are device pointers on the evaluator's device, d_cost is one double.
 * Asynchronous on the evaluator's stream; call cse_wait for the status. */
int cse_evaluate_device(cse_evaluator* ev, const double* d_state, double* d_cost,
                        double* d_residuals, double* d_gradient,
                        double* d_jacobian_values);

/* Evaluate flags.  CSE_EVAL_SAME_POINT carries
 * Evaluator::EvaluateOptions::new_evaluation_point == false
 * (internal/ceres/evaluator.h:106-107): the state has the same values as at
 * the previous evaluation on this evaluator, as when TrustRegionMinimizer
 * evaluates the Jacobian at a just-accepted candidate
 * (trust_region_minimizer.cc:822-826).  The library then reuses what it
 * derived from the state last time: the state already copied to the device
 * (cse_evaluate_ex, the multi-device evaluator) and the repacked slot-0
 * table of the affine kernels.  The state pointer may differ; its values
 * must not.  Ignored when there is no previous evaluation to reuse. */
#define CSE_EVAL_SAME_POINT 1u

/* cse_evaluate / cse_evaluate_device with flags (0 = the plain call). */
int cse_evaluate_ex(cse_evaluator* ev, const double* state, double* cost,
                    double* residuals, double* gradient, double* jacobian_values,
                    uint32_t flags);
int cse_evaluate_device_ex(cse_evaluator* ev, const double* d_state, double* d_cost,
                           double* d_residuals, double* d_gradient,
                           double* d_jacobian_values, uint32_t flags);

/* ---- User functor kinds -------------------------------------------------
 * The reference evaluates any AutoDiffCostFunction functor: the user's nvcc
 * TU instantiates EvaluateKernel<CostFunctor, LossFunctionCUDA, kR, Ns...>
 * and ProblemCUDA::AddResidualBlock registers one
 * AutoDiffResidualBlockCUDAEvaluator per such type
 * (include/ceres/problem_cuda.h:423-474, README.md:19-33).  Here the user's
 * hipcc TU instantiates this library's kernels for its functor
 * (include/ceres_amd/autodiff_cuda.h, header-only: RegisterAutoDiffFunctor
 * or ProblemCUDA::AddResidualBlock) and registers them as a table of launch
 * functions; the kind returned is then used in cse_residual_group.
 * functor_kind like a built-in one.  Kinds are process-wide and stay
 * registered until the library is unloaded.
 *
 * The launch functions receive the library's kernel argument blocks, whose
 * layout both sides take from the same headers (ceres-solver-cuda_amd/csrc/
 * kernel_common.hpp, operator_kernels.hpp); kernel_args_size, gradient_args_size
 * and kernel_args_tag must equal the library's or registration fails. */
#define CSE_FUNCTOR_USER_FIRST 1000
#define CSE_MAX_PARAMETER_BLOCKS 10

/* Evaluation: kernel_args -> the group's arguments, stream = hipStream_t. */
typedef void (*cse_kernel_launch_fn)(const void* kernel_args, int64_t num_workgroups, void* stream);
/* which: 0 = y += J x on the affine layout, 1 = y += J x (general),
 * 2 = y += J^T x (general). */
typedef void (*cse_multiply_launch_fn)(const void* kernel_args, int32_t which, const double* x,
                                       double* y, void* stream);
/* The gradient post-pass of one slot; form 0 = identity order, 1 = chunked,
 * 2 = one lane per parameter block. */
typedef void (*cse_gradient_launch_fn)(const void* gradient_args, const void* chunks, int32_t form,
                                       void* stream);
/* The fused gradient's slot-0 rows: one wave per chunk of a slot-0 block's
 * residual blocks, re-evaluated in slot-0 order (camera_gradient_args ->
 * the library's CamGradArgs); num_slots = waves to launch. */
typedef void (*cse_camera_gradient_launch_fn)(const void* camera_gradient_args, int64_t num_slots,
                                              void* stream);

typedef struct cse_functor_ops {
  int32_t abi_version;          /* CSE_ABI_VERSION */
  int32_t num_residuals;        /* kNumResiduals */
  int32_t num_parameter_blocks; /* sizeof...(Ns) */
  int32_t parameter_block_sizes[CSE_MAX_PARAMETER_BLOCKS];
  int32_t data_size;            /* doubles of functor data per residual block */
  int32_t loss_kind;            /* the cse_loss_kind the kernels apply; groups must match */
  int32_t loss_size;            /* CSE_LOSS_USER: bytes of the loss object */
  int32_t kernel_args_size;
  int32_t gradient_args_size;
  int32_t camera_gradient_args_size; /* with camera_gradient; else 0 */
  int32_t reserved;             /* 0 */
  uint64_t kernel_args_tag;
  const char* name;             /* copied; for messages and cse_functor_name */
  cse_kernel_launch_fn table[2];        /* general kernel [0 residuals/cost, 1 + Jacobian] */
  cse_kernel_launch_fn affine[2][2][2]; /* [CompressedRow][Jacobian][LDS-DMA gather]; NULL = none */
  cse_multiply_launch_fn multiply;
  cse_gradient_launch_fn gradient[2];   /* per slot of an affine kind; NULL = in-kernel atomics */
  /* ABI 5, two-slot affine kinds whose slot 1 has 3 parameters (both or
   * neither): gradient_mode 0's fused form, as the library's Snavely kinds
   * take it -- the Jacobian kernel that also sums the slot-1 rows
   * [CompressedRow], and the slot-0 rows by re-evaluation.  NULL = the
   * gradient post-passes above. */
  cse_kernel_launch_fn fused_points[2];
  cse_camera_gradient_launch_fn camera_gradient;
} cse_functor_ops;

/* Registers a user functor kind; *kind receives its number
 * (>= CSE_FUNCTOR_USER_FIRST).  Registering the same table again (same name,
 * shape and launch functions) returns the same kind. */
int cse_register_functor(const cse_functor_ops* ops, int32_t* kind);

/* Shape of a built-in or registered kind; parameter_block_sizes receives
 * *num_parameter_blocks entries (room for CSE_MAX_PARAMETER_BLOCKS). */
int cse_functor_shape(int32_t kind, int32_t* num_residuals, int32_t* num_parameter_blocks,
                      int32_t* parameter_block_sizes, int32_t* data_size);

/* Synchronises the evaluator's stream and returns the status of the most
 * recent evaluation (CSE_OK / CSE_EVALUATION_FAILED) or an error. */
int cse_wait(cse_evaluator* ev);

/* Replaces RegisteredCUDAEvaluators::UpdatePlusJacobians
 * (registered_cuda_evaluators.cc:105-121): host array of
 * num_plus_jacobian_values doubles. */
int cse_set_plus_jacobians(cse_evaluator* ev, const double* plus_jacobians);

/* Replaces Evaluator::Plus -> Program::Plus (internal/ceres/program.cc:121-149,
 * internal/ceres/parameter_block.h:227-251) for problems whose active
 * parameter blocks have no manifold or the quaternion manifold:
 * x_plus_delta = x + delta block by block (state offsets vs delta offsets of
 * the descriptor), CSE_MANIFOLD_QUATERNION_EUCLIDEAN blocks by their
 * manifold's Plus.  Box constraints are not part of the descriptor, so none
 * are applied.  Returns CSE_ERR_UNSUPPORTED when an active block has an
 * explicit plus-Jacobian manifold (the caller keeps Ceres' host Plus).
 *   cse_plus_device: device pointers, asynchronous on the evaluator's stream
 *   cse_plus:        host pointers, synchronous */
int cse_plus_device(cse_evaluator* ev, const double* d_state, const double* d_delta,
                    double* d_state_plus_delta);
int cse_plus(cse_evaluator* ev, const double* state, const double* delta,
             double* state_plus_delta);

/* The Jacobian as a linear operator on the device (a consumer of
 * the evaluator's output that keeps it in HBM).  J is d_jacobian_values as
 * this evaluator writes it (the descriptor's BlockSparse or CompressedRow
 * layout); x and y are device vectors; asynchronous on the evaluator's
 * stream.
 *   cse_jacobian_right_multiply: y += J x  (x: num_effective_parameters,
 *       y: num_residuals) -- CudaSparseMatrix::RightMultiplyAndAccumulate
 *       (internal/ceres/cuda_sparse_matrix.h:77), BlockSparseMatrix::
 *       RightMultiplyAndAccumulate (block_sparse_matrix.h:76)
 *   cse_jacobian_left_multiply:  y += J^T x (x: num_residuals,
 *       y: num_effective_parameters) -- LeftMultiplyAndAccumulate
 *       (cuda_sparse_matrix.h:79, block_sparse_matrix.h:81); deterministic on
 *       the affine path (per-parameter-block ordered sums), FP64 atomics on
 *       the table path.
 * The reference copies the values to the host and back (CopyValuesFromCpu,
 * cuda_sparse_matrix.h:96); here they never leave HBM. */
int cse_jacobian_right_multiply(cse_evaluator* ev, const double* d_jacobian_values,
                                const double* d_x, double* d_y);
int cse_jacobian_left_multiply(cse_evaluator* ev, const double* d_jacobian_values,
                               const double* d_x, double* d_y);

/* The CGNR normal operator: y += J^T (J x) + D .* D .* x (d_D may be NULL),
 * device pointers, asynchronous on the evaluator's stream.  Replaces
 * CudaCgnrLinearOperator::RightMultiplyAndAccumulate
 * (internal/ceres/cgnr_solver.cc:226-237: z = A x, y += A^T z, y.DtDxpy(D, x)).
 * Groups eligible for the fused gradient (cse_info.num_fused_gradient_groups)
 * read J once and never materialise z; otherwise the two products above.
 * Deterministic on the affine path. */
int cse_cgnr_multiply(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D,
                      const double* d_x, double* d_y);

/* ---- ITERATIVE_SCHUR on the device -------------------------------------
 * The implicit Schur complement of the Jacobian this evaluator wrote, for
 * the linear solve of a Schur-ordered bundle adjustment problem: replaces
 * ImplicitSchurComplement (internal/ceres/implicit_schur_complement.h:
 * 86-160) and the preconditioners IterativeSchurComplementSolver builds
 * (iterative_schur_complement_solver.cc:172-204).  With the Jacobian
 * A = [E F] (e blocks = the points, slot 1; f blocks = the cameras, slot 0),
 * a per-column diagonal D and the right-hand side b, the system
 * (A^T A + D^2) [y_e; y_f] = A^T b is reduced to
 *     S y_f = rhs,  S = F^T F + D_f^2 - F^T E (E^T E + D_e^2)^-1 E^T F,
 *     rhs = F^T (b - E (E^T E + D_e^2)^-1 E^T b).
 * Requires (CSE_ERR_UNSUPPORTED otherwise) one group of the Snavely shape
 * (2 residuals, a camera of 9 tangent parameters, a point of 3: the
 * library's Snavely kinds or a user kind; the operators read only the
 * Jacobian) on the affine BlockSparseMatrix path whose points occupy the effective columns
 * [0, num_cols_e) and cameras the rest, as ITERATIVE_SCHUR's elimination
 * ordering gives.  All device pointers, asynchronous on the evaluator's
 * stream, deterministic. */
enum cse_schur_preconditioner {
  CSE_SCHUR_IDENTITY = 0,     /* IDENTITY: M^-1 = I */
  CSE_SCHUR_JACOBI = 1,       /* JACOBI: block diagonal (F^T F + D_f^2)^-1 */
  CSE_SCHUR_SCHUR_JACOBI = 2  /* SCHUR_JACOBI: block diagonal of S, inverted
                                 (schur_jacobi_preconditioner.cc:89-98) */
};

/* The column split: num_cols_e (points) and num_cols_f (cameras). */
int cse_schur_structure(cse_evaluator* ev, int64_t* num_cols_e, int64_t* num_cols_f);

/* ImplicitSchurComplement::Init(A, D, b) (implicit_schur_complement.cc:
 * 53-99) plus Preconditioner::Update: binds d_jacobian_values, d_D
 * (num_effective_parameters entries, may be NULL) and d_b (num_residuals)
 * -- they must stay valid until the next init -- computes the per-point
 * (E^T E + D_e^2)^-1, writes rhs (num_cols_f) and builds the preconditioner.
 * With d_D NULL a block can be singular (a point seen by one residual block,
 * a camera without observations): a Cholesky pivot that is not positive
 * leaves that block's inverse zero and makes the next cse_wait return
 * CSE_EVALUATION_FAILED, where Eigen's LLT would spread NaN silently. */
int cse_schur_init(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D,
                   const double* d_b, double* d_rhs, int preconditioner);

/* cse_schur_init, and also the gradient g = J^T r of the bound Jacobian into
 * d_gradient (num_effective_parameters entries, assigned), taking r = -b --
 * the trust-region step's b (TrustRegionMinimizer::EvaluateGradientAndJacobian
 * evaluates g = J^T r beside J, trust_region_minimizer.cc:242-255) -- in the
 * same passes over J: the e rows from the E^T b sums the init forms anyway,
 * the f rows -F^T b in the camera-order pass that forms F^T u and the
 * preconditioner, from b_b stored beside u_b.  Then the evaluation before it
 * needs no gradient (no CameraGradientKernel).  Deterministic; equals the
 * evaluation's gradient (gradient_mode 0) to rounding (a different
 * summation order). */
int cse_schur_init_gradient(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D,
                            const double* d_b, double* d_rhs, int preconditioner,
                            double* d_gradient);

/* y = S x (ImplicitSchurComplement::RightMultiplyAndAccumulate, :101-141,
 * which assigns y); x and y have num_cols_f entries. */
int cse_schur_multiply(cse_evaluator* ev, const double* d_x, double* d_y);

/* y += M^-1 x for the preconditioner chosen at init. */
int cse_schur_precondition(cse_evaluator* ev, const double* d_x, double* d_y);

/* ImplicitSchurComplement::BackSubstitute(x, y) (:216-238): y
 * (num_effective_parameters) = [(E^T E + D_e^2)^-1 E^T (b - F x); x]. */
int cse_schur_back_substitute(cse_evaluator* ev, const double* d_x, double* d_y);

/* ---- One host solve, several GPUs --------------------------------------
 * The reference evaluates on one device (ContextImpl's single stream,
 * include/ceres/internal/cuda_buffer.h:98) and Ceres' host solve calls one
 * RegisteredCUDAEvaluators::Evaluate with host pointers
 * (include/ceres/internal/registered_cuda_evaluators.h:75-79).
 * cse_create_multi builds such an evaluator over several devices (SURVEY.md
 * §8(b) "device list", §8(e)): the residual blocks are cut into num_devices
 * contiguous shards at point-bucket boundaries (a block whose last parameter
 * block differs from the previous block's; multiples of 4 blocks where
 * possible), each shard is evaluated on devices[k] (repeats allowed: several
 * shards on one device) holding only the parameter blocks its residual blocks
 * use (a BAL shard: every camera it sees plus its own point slice), and
 * cse_evaluate on the returned handle
 *   - copies each shard's slices of the state to its device (only those
 *     slices: cse_shard_transfer_bytes);
 *   - copies each shard's residual and Jacobian-value strips straight into
 *     disjoint regions of the caller's one residuals / jacobian_values
 *     buffers, concurrently per device when the buffers are page-locked
 *     (cse_host_register, or the caller's own hipHostMalloc), synchronously
 *     otherwise -- the library never pins a caller buffer by itself;
 *   - sums the cost and the gradient over the shards in shard order on the
 *     host (deterministic; a parameter block used by several shards, e.g. a
 *     camera, gets the sum of their rows).
 * On an error every copy already queued is finished before the call returns.
 * options->use_stream and options->stream must be 0 (each device gets its
 * own stream).  On such a handle cse_evaluate, cse_wait (returns CSE_OK),
 * cse_plus, cse_set_plus_jacobians, cse_get_info (sizes of the whole
 * problem; bytes summed over the shards), cse_kernel_stats (the slowest
 * shard), cse_shard_info, cse_shard_transfer_bytes and cse_destroy work; the
 * device-pointer entry points return CSE_ERR_UNSUPPORTED. */
int cse_create_multi(const cse_problem_desc* desc, const cse_options* options,
                     const int32_t* devices, int32_t num_devices, cse_evaluator** out);

/* The shards of an evaluator: *num_shards; first_block[num_shards + 1] (may be
 * NULL) = the residual-block ranges [first_block[k], first_block[k+1]);
 * devices[num_shards] (may be NULL).  A cse_create evaluator has one shard. */
int cse_shard_info(cse_evaluator* ev, int32_t* num_shards, int64_t* first_block,
                   int32_t* devices);

/* Bytes one cse_evaluate moves per shard: state_h2d_bytes[num_shards] (the
 * state slices the shard's device receives), strips_d2h_bytes[num_shards]
 * (its residual and Jacobian-value strips); either may be NULL.  A cse_create
 * evaluator has one shard (the whole state and outputs). */
int cse_shard_transfer_bytes(cse_evaluator* ev, int64_t* state_h2d_bytes,
                             int64_t* strips_d2h_bytes);

/* Page-locks [p, p + bytes) of the caller's memory (hipHostRegister) for
 * asynchronous copies until cse_host_unregister(p) with the same p; the
 * multi-device evaluator then copies state slices and strips to and from
 * buffers inside the range without staging.  The caller owns the range:
 * unregister before freeing it.  (The reference pins inside its ContextImpl
 * buffers, include/ceres/internal/cuda_buffer.h:98; here the caller's Ceres
 * arrays are the transfer buffers.) */
int cse_host_register(void* p, size_t bytes);
int cse_host_unregister(void* p);

void cse_destroy(cse_evaluator* ev);

/* Thread-local description of the last error. */
const char* cse_last_error(void);

typedef struct cse_info {
  int64_t num_residual_blocks;
  int64_t num_residuals;
  int64_t num_parameters;
  int64_t num_effective_parameters;
  int64_t num_jacobian_values;
  int32_t num_groups;
  int32_t num_affine_groups;  /* groups on the table-free fast path */
  int32_t device;
  int32_t num_fused_gradient_groups; /* groups whose gradient is fused into the
                                        evaluation (options.gradient_mode 0) */
  /* Compulsory HBM bytes of one residual+Jacobian evaluation (SURVEY.md
   * §8(d)): per block functor data + parameter ids + residuals + Jacobian
   * values, plus each distinct parameter block read once. */
  int64_t bytes_jacobian_eval;
  int64_t bytes_residual_eval; /* same without the Jacobian values */
} cse_info;

int cse_get_info(cse_evaluator* ev, cse_info* info);

/* Kernel time of the evaluate kernels (HIP events on the evaluator's
 * stream, needs options.profile): last launch and running totals. */
int cse_kernel_stats(cse_evaluator* ev, double* last_ms, double* total_ms,
                     int64_t* launches);
int cse_reset_kernel_stats(cse_evaluator* ev);

/* Host-side layout builders for callers that do not have Ceres' writers
 * (restating internal/ceres/block_jacobian_writer.cc:62-160 and
 * compressed_row_jacobian_writer.cc:93-193,240-300).
 *
 * Inputs: parameter blocks (program order) and, per residual block in
 * program order, its parameter block ids (CSR: param_begin[nrb+1]) and
 * residual count.  Outputs the residual layout, per-residual layout and
 * offsets (sized by the *_count queries) and the value count.  For CRS,
 * crs_rows[num_residuals+1] and crs_cols[num_values] are optional. */
int cse_block_sparse_layout(int64_t num_parameter_blocks,
                            const cse_parameter_block* parameter_blocks,
                            int64_t num_residual_blocks, const int64_t* param_begin,
                            const int32_t* param_ids, const int32_t* num_residuals,
                            int64_t num_eliminate_blocks, int64_t* residual_layout,
                            int64_t* jacobian_per_residual_layout,
                            int64_t* jacobian_per_residual_offsets,
                            int64_t* num_jacobian_values);
int cse_compressed_row_layout(int64_t num_parameter_blocks,
                              const cse_parameter_block* parameter_blocks,
                              int64_t num_residual_blocks, const int64_t* param_begin,
                              const int32_t* param_ids, const int32_t* num_residuals,
                              int64_t* residual_layout,
                              int64_t* jacobian_per_residual_layout,
                              int64_t* jacobian_per_residual_offsets,
                              int64_t* num_jacobian_values, int64_t* crs_rows,
                              int64_t* crs_cols);
/* Number of jacobian_per_residual_offsets entries for either layout. */
int64_t cse_layout_offsets_count(int64_t num_parameter_blocks,
                                 const cse_parameter_block* parameter_blocks,
                                 int64_t num_residual_blocks, const int64_t* param_begin,
                                 const int32_t* param_ids, const int32_t* num_residuals);

/* Library identification: ABI version and the gfx target it was built for. */
int cse_abi_version(void);
const char* cse_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* CSE_H_ */
