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
  return 0;
}
