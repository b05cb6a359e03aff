set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --path of > gpurun_out/r2_bench_of.json 2> gpurun_out/r2_bench_of.err
timeout -k 10 300 python3 -u bench.py > gpurun_out/r2_bench_fd.json 2> gpurun_out/r2_bench_fd.err
bash tools/profile_round.sh r2of of_1080p_single_feed_per_gpu --path of
bash tools/profile_round.sh r2fd fd_1080p_single_feed_per_gpu
