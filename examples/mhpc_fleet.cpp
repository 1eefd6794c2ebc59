// A fleet of controllers in one batch, each at its own gait point (SURVEY.md 8 north_star:
// the batch axis over initial states / gait schedules).  In the reference every controller is
// its own MHPCLocomotion, built from its own Gait at its current mode (MHPCLocomotion.cpp
// :63-104) and advanced by its own update_problem (:107-158).  Here one handle holds them
// all: problem b gets layout b % 6 -- the PRONK / default-branch 2 WB + 2 SRB controller at
// each of its four modes and the BOUND 4 WB + 6 SRB controller at modes 1 and 3 -- then
// every second controller advances one gait step and the batch is solved again.
// Prints one line per problem and solve: "solve s problem b layout l J = ... modes m/N ...".
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mhpc_locomotion.hpp"

int main(int argc, char** argv) {
  const int batch = argc > 1 ? std::atoi(argv[1]) : 12;
  HSDDP_OPTION<double> option;
  option.max_AL_iter = 2;
  option.max_DDP_iter = 3;
  USRCMD usrcmd{1.5f, 0.f, 0.f, 0.f, 0.f};
  Gait pronk(GaitType2D::PRONK), bound;
  MHPCUserParameters trot_p, bound_p;
  trot_p.n_wbphase = 2; trot_p.n_fbphase = 2; trot_p.usrcmd = &usrcmd;
  bound_p.n_wbphase = 4; bound_p.n_fbphase = 6; bound_p.usrcmd = &usrcmd;
  std::vector<mhpc_problem_desc> layouts;
  for (int c = 1; c <= 4; ++c) {
    trot_p.cmode = c;
    layouts.push_back(MHPCLocomotion<double>::build_desc(&trot_p, &pronk));
  }
  for (int c : {1, 3}) {
    bound_p.cmode = c;
    layouts.push_back(MHPCLocomotion<double>::build_desc(&bound_p, &bound));
  }
  std::vector<int32_t> layout_of(batch), gait_of(batch), steps(batch);
  for (int b = 0; b < batch; ++b) {
    layout_of[b] = b % 6;
    gait_of[b] = layout_of[b] < 4 ? 0 : 1;
    steps[b] = b % 2;
  }
  trot_p.cmode = 1;
  MHPCLocomotion<double> fleet(&trot_p, &pronk, option, batch);
  fleet.set_layouts(layouts, layout_of);
  fleet.initialization();
  for (int s = 0; s < 2; ++s) {
    if (s == 1) fleet.update_problems({&pronk, &bound}, gait_of, steps);
    fleet.solve_mhpc();
    for (int b = 0; b < batch; ++b) {
      fleet.select_problem(b);
      const mhpc_problem_desc& d = fleet.desc();
      std::printf("solve %d problem %d layout %d J = %.17g phases %zu modes", s, b, layout_of[b],
                  fleet._actual_cost, fleet._phases.size());
      for (int p = 0; p < d.n_wb + d.n_fb; ++p) std::printf(" %d/%d", d.mode_seq[p], d.N[p]);
      std::printf("\n");
    }
  }
  std::printf("layouts in use: %d\n", fleet.num_layouts());
  return 0;
}
