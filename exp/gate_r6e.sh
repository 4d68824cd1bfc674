tools/gpu_gate.sh r6e && tools/profile_sq_pair.sh r6e && exp/pmc_train_kernels.sh r6e_c5
