// Receding-horizon MPC loop on the reference's controller surface:
// initialization + solve_mhpc, then every tick the robot is assumed to follow the plan
// perfectly up to the end of the first phase, that state becomes the new initial condition,
// update_problem() shifts the horizon (gait advances one mode, phase buffers rotate as warm
// start) and solve_mhpc() runs again.  Prints cost and phase layout per tick.
#include <cstdio>
#include <vector>

#include "mhpc_locomotion.hpp"

int main(int argc, char** argv) {
  const int ticks = argc > 1 ? std::atoi(argv[1]) : 5;
  HSDDP_OPTION<double> option;
  option.max_AL_iter = 2;
  option.max_DDP_iter = 3;
  USRCMD usrcmd{1.5f, 0.f, 0.f, 0.f, 0.f};
  MHPCUserParameters params;  // 4 WB + 4 SRB phases, as test_main.cpp
  params.usrcmd = &usrcmd;
  Gait gait;  // BOUND
  MHPCLocomotion<double> loco(&params, &gait, option);
  loco.initialization();
  for (int t = 0; t < ticks; ++t) {
    if (t > 0) loco.update_problem();
    loco.solve_mhpc();
    const mhpc_problem_desc& d = loco.desc();
    std::printf("tick %d J = %.9g  viol = %.3g  modes", t, loco._actual_cost,
                loco._tconstr_violation);
    for (int p = 0; p < d.n_wb + d.n_fb; ++p) std::printf(" %d/%d", d.mode_seq[p], d.N[p]);
    std::printf("\n");
    // the state at the end of phase 0 of the plan is where the robot will be next tick
    MHPCLocomotion<double>::ExecHorizon e = loco.get_exec();
    const int k = d.N[0] - 1;
    std::vector<double> x0(e.x.begin() + (size_t)k * 14, e.x.begin() + (size_t)(k + 1) * 14);
    loco.set_initial_condition(x0);
  }
  return 0;
}
