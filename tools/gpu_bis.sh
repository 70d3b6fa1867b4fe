#!/bin/bash
# bisect: the same few GPU tests against libraries built from earlier commits (SOARM_SIM_LIB)
mkdir -p gpurun_out
K="test_one_substep_with_contacts or test_newton_solver_contact_free or odd_batch_sizes or test_one_substep_no_contact"
for c in 1469c2c 7671766 9367ba9 a551c5c current; do
  lib=tools/_bis/lib_$c.so
  [ $c = current ] && lib=lerobot-mujoco-sim2real_amd/csrc/libsoarm_sim.so
  SOARM_SIM_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "$K" --timeout 120 --timeout-method thread > gpurun_out/bis_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc $(tail -1 gpurun_out/bis_$c.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
