set -u
cd $GRAFT_REPO_ROOT
for m in 4096 512 128; do
TDE_PYR_MAXB=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_pyr$m" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_pyr$m.log 2>&1 || exit $?
echo "$m $(grep -h 'depth_pyramid' $(find gpurun_out/prof_pyr$m -name '*kernel_stats.csv') | cut -d, -f3-4)"
done
