# validate.sh, configs.sh, then scale_n.sh:
#   gpurun --timeout 1500 -- bash bench/gpu_runs/all.sh <tag>
bash bench/gpu_runs/validate.sh ${1:-all} 100 && bash bench/gpu_runs/configs.sh ${1:-all}_configs \
    && bash bench/gpu_runs/scale_n.sh ${1:-all}_scale_n
