#!/bin/bash
# build the current csrc into tools/_ab/lib_$1.so (A/B comparisons via SOARM_SIM_LIB);
# extra arguments are passed to hipcc (e.g. -DSOME_SWITCH)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/tools/_ab
read FLAGS SRCS <<< "$(cd $R && python -c "
import soarm_pkg, os
from lerobot_mujoco_sim2real_amd.build import FLAGS, SOURCES, SRC_DIR
print(' '.join(FLAGS).replace(' ', ',') + ' ' + ','.join(os.path.join(SRC_DIR, f) for f in SOURCES))")"
N=$1; shift
/opt/rocm/bin/hipcc ${FLAGS//,/ } "$@" -o $R/tools/_ab/lib_$N.so ${SRCS//,/ }
