// Per-precision implementation of the C-ABI (mhpc_runtime.cpp compiled once per arithmetic
// type into namespace API_NS); mhpc_capi.cpp exports the extern "C" symbols and dispatches
// on the descriptor's precision.  No include guard: included once per namespace.
namespace API_NS {
struct Handle;
const char* api_kernel_name(int k);
int api_create(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt, int batch, int device,
               Handle** out);
int api_set_x0(Handle* h, const double* x0);
int api_initialize(Handle* h);
int api_solve(Handle* h, int32_t* status);
int api_get_phase(Handle* h, int phase, int first, int count, double* x, double* u, double* y,
                  double* K, double* du, double* Vx);
int api_batch(Handle* h);
int api_get_scalars(Handle* h, double* J, double* dV_exp, double* viol, double* V_phase,
                    double* dV_phase, int32_t* trace);
int api_rollout_costs(Handle* h, int n_eps, const double* eps, double* J, double* viol, float* ms);
int api_get_cost_gradients(Handle* h, int phase, int first, int count, double* lx, double* Phix);
int api_update_problem(Handle* h, const mhpc_gait* gait);
int api_update_problems(Handle* h, int n_gaits, const mhpc_gait* gaits, const int32_t* gait_of,
                        const int32_t* steps);
int api_set_layouts(Handle* h, int n_desc, const mhpc_problem_desc* descs, const int32_t* lop);
int api_get_problem_desc(Handle* h, int b, mhpc_problem_desc* desc);
int api_num_layouts(Handle* h, int* n);
int api_max_phases(Handle* h, int* n);
int api_get_desc(Handle* h, mhpc_problem_desc* desc);
int api_get_counters(Handle* h, mhpc_counters* c);
int api_set_profiling(Handle* h, int on);
int api_get_kernel_stats(Handle* h, double* ms, int64_t* launches, double* alg_bytes);
int api_reset_kernel_stats(Handle* h);
int api_get_kernel_flops(Handle* h, double* flops);
int api_set_kernel_variant(Handle* h, int which, int variant);
int api_set_cost_weights(Handle* h, const mhpc_cost_weights* w);
int api_get_cost_weights(Handle* h, mhpc_cost_weights* w);
int api_set_constraint_params(Handle* h, const mhpc_constraint_params* c);
int api_get_constraint_params(Handle* h, mhpc_constraint_params* c);
void api_destroy(Handle* h);
}  // namespace API_NS
