// options.h — per-handle tuning and verification options (pfe_set_option, include/pfe.h).
//
// The defaults are the product configuration.  Nothing in the library reads the process
// environment: a stray variable can never change the scores a caller gets.
#pragma once

#include "../../include/pfe.h"

namespace pfe {

struct Options {
  int solver = PFE_SOLVER_POOLED;  // LM solver of the 22-score kernels
  int serial = 0;                  // 1: score groups in order on the handle's stream
  int handover = 1;                // 0: re-evaluate the function after accepted LM steps
  int gslots = 0;                  // fit slots per pooled wave (0: sized from n and the CUs)
  int lyon8_blocks = 131072;       // grid cap of the Lyon-8 stream kernel
  int lyon8_burst = 2;             // candidate groups per wave step of the Lyon-8 kernel
  int pfd_waves = 4;               // waves per fold of the PFD dmprof kernel (4 or 1)
  int lyon8_dm = 0;                // DataBlock DM rows (pfe.h PFE_OPT_LYON8_DM, 0..2)
  int pfd_split = 0;               // PFD dmprof: 1 part sums by k_pfd_parts beside the sweep, 0 fused
  int lyon8_dm_split = 1;          // DataBlock rows: 1 split last chunks + paired one-chunk rows,
                                   // 2 chain splits only, 0 one lane per leaf
};

}  // namespace pfe
