set -o pipefail
mkdir -p gpurun_out
python -c "import bench; print(bench.host_threads())" > gpurun_out/r3_cpu_threads.log 2>&1
timeout -k 10 1100 python -u bench.py --cpu-plan > gpurun_out/r3_cpu_plan.log 2> gpurun_out/r3_cpu_plan.err
