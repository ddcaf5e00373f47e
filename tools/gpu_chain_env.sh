bash tools/gpu_chainw.sh r21_chainw9 && bash tools/gpu_envelope_n100.sh env_n100_a 7
