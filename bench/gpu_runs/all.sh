# validate.sh then configs.sh: gpurun --timeout 1500 -- bash bench/gpu_runs/all.sh <tag>
bash bench/gpu_runs/validate.sh ${1:-all} 100 && bash bench/gpu_runs/configs.sh ${1:-all}_configs
