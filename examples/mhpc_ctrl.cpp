// The reference's demo driver (test_main.cpp:12-35), compiled against this framework's
// C++ surface: same option / parameter / gait objects, same three calls.  Optional
// argument: batch size (independent problems solved at once on GPU 0).
#include <cstdio>
#include <cstdlib>

#include "mhpc_locomotion.hpp"

int main(int argc, char* argv[]) {
  // Choose HSDDP options
  HSDDP_OPTION<double> option;
  option.ReB_active = 1;
  option.AL_active = 1;
  option.max_AL_iter = 2;
  option.max_DDP_iter = 3;

  // Instantiate MHPCLocomotion
  USRCMD usrcmd;
  usrcmd.vel = 1.5;
  usrcmd.height = 0;
  usrcmd.roll = 0;
  usrcmd.pitch = 0;
  usrcmd.yaw = 0;
  MHPCUserParameters mhpcparams;
  mhpcparams.usrcmd = &usrcmd;
  Gait gait;
  const int batch = argc > 1 ? std::atoi(argv[1]) : 1;
  MHPCLocomotion<double> locomotion(&mhpcparams, &gait, option, batch);
  locomotion.initialization();
  locomotion.solve_mhpc();
  locomotion.print_debugInfo();
  std::printf("J = %.9g  dV = %.6g  violation = %.6g  status = %d\n", locomotion._actual_cost,
              locomotion._exp_cost_change, locomotion._tconstr_violation,
              locomotion.status()[0]);

  // Per-phase results through the reference's public phase interface
  // (SinglePhaseAbstract.h:79-81,116-119), as MHPCLocomotion::solve_mhpc reads them
  // (MHPCLocomotion.cpp:178-194): phases.txt, one header line per phase, then one line per knot
  // with x, u, y, G, du, K (row-major 4 x xsize), for a test to compare with the oracle.
  FILE* f = std::fopen("phases.txt", "w");
  for (int p = 0; p < locomotion._n_phases; ++p) {
    SinglePhaseAbstract<double>* ph = locomotion._phases[p];
    std::fprintf(f, "phase %d mode %d N %zu V %.17g dV %.17g\n", ph->_phaseidx,
                 (int)ph->get_modeidx(), ph->_N_TIMESTEPS, ph->_V, ph->_dV);
    auto dump = [&](auto* ms, auto* ctg) {
      const size_t n = ms[0].x.size();
      for (size_t k = 0; k < ph->_N_TIMESTEPS; ++k) {
        for (size_t i = 0; i < n; ++i) std::fprintf(f, "%.17g ", ms[k].x(i));
        for (size_t i = 0; i < 4; ++i) std::fprintf(f, "%.17g ", ms[k].u(i));
        for (size_t i = 0; i < 4; ++i) std::fprintf(f, "%.17g ", ms[k].y(i));
        for (size_t i = 0; i < n; ++i) std::fprintf(f, "%.17g ", ctg[k].G(i));
        for (size_t i = 0; i < 4; ++i) std::fprintf(f, "%.17g ", ctg[k].du(i));
        for (size_t r = 0; r < 4; ++r)
          for (size_t j = 0; j < n; ++j) std::fprintf(f, "%.17g ", ctg[k].K(r, j));
        std::fprintf(f, "\n");
      }
    };
    if (ph->_xsize == 14)
      dump((ModelState<double, 14, 4, 4>*)ph->get_nominal_ms_ptr(),
           (CostToGoStruct<double, 14, 4>*)ph->get_CTG_info_ptr());
    else
      dump((ModelState<double, 6, 4, 4>*)ph->get_nominal_ms_ptr(),
           (CostToGoStruct<double, 6, 4>*)ph->get_CTG_info_ptr());
  }
  std::fclose(f);
  return 0;
}
