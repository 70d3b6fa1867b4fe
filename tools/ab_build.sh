#!/bin/bash
# build the current csrc into tools/_ab/lib_$1.so (A/B comparisons via SOARM_SIM_LIB)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/tools/_ab
FLAGS=$(cd $R && python -c "import soarm_pkg; from lerobot_mujoco_sim2real_amd.build import FLAGS; print(' '.join(FLAGS))")
/opt/rocm/bin/hipcc $FLAGS -o $R/tools/_ab/lib_$1.so $R/lerobot-mujoco-sim2real_amd/csrc/soarm_sim.hip
