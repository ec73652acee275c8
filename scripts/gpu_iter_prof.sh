set -u
bash scripts/gpu_iter.sh it3 && bash scripts/profile.sh
