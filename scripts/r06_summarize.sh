#!/bin/bash
# CPU side, after `scripts/r06_collect.sh a` and `b` ran on the GPU box: turn gpurun_out/ into the
# stamped summaries under profiles/ (the bench attaches them only when their src_sha256 matches).
set -e
G=gpurun_out; P=profiles
cp $G/pmc_lk/pmc_lk.json $P/pmc_lk_iter.json
python3 scripts/pmc_step_to_json.py $G/pmc_step $P/pmc_step.json > /dev/null
python3 scripts/pmc_to_json.py $G/pmc_warp 3840x2160x32 $P/pmc_warp_diff.json > /dev/null
python3 scripts/pmc_warp_summary.py $G/pmc_warpc > $P/r06_pmc_warp_counters.txt
python3 scripts/kt_warp_to_json.py $G/r06/warp_kt 3840x2160x32 $P/warp_kernel_trace.json 20 > /dev/null
python3 scripts/kt_warp_to_json.py $G/r06/warp_kt_proj 3840x2160x32 $P/warp_kernel_trace_projective.json 20 > /dev/null
python3 scripts/summarize_prof.py $(find $G/r06/warp_kt -name run_kernel_trace.csv) "warp roofline leg (affine), kernel records" > $P/r06_warp_kernel_trace.md
python3 scripts/summarize_prof.py $(find $G/r06/warp_kt_proj -name run_kernel_trace.csv) "warp roofline leg (projective), kernel records" > $P/r06_warp_kernel_trace_projective.md
python3 scripts/summarize_prof.py $G/prof_r06/run_kernel_trace.csv "default bench (1080p x 32, pipelined), kernel records" > $P/r06_kernel_trace.md
cp $G/prof_r06/run_kernel_stats.csv $P/r06_kernel_stats.csv; cp $G/prof_r06/bench_stdout.json $P/r06_prof_bench.json
python3 scripts/pipe_timeline.py $G/prof_r06/run_kernel_trace.csv > $P/r06_pipe_timeline.txt
python3 scripts/summarize_prof.py $(find $G/r06/live/kt -name run_kernel_trace.csv) "live leg (5 x 1080p rgb8 ring callback + fitSubspace), kernel records" > $P/r06_live_kernel_trace.md
cp $G/r06/lk_tail.txt $P/r06_lk_tail.txt; cp $G/r06/lk_levels.txt $P/r06_lk_levels.txt
cp $G/r06/pytest_gpu.log $P/r06_pytest_gpu.txt; cp $G/r06/smoke.txt $P/r06_smoke.txt
cp $G/r06/c4_n1_k8_f2.json $P/r06_c4_n1_k8_f2.json; cp $G/r06/c4_n1_k1_f2.json $P/r06_c4_n1_k1_f2.json
grep '^{' $G/r06/c4_n2_k8_f2.json > $P/r06_c4_n2_k8_f2.json; cp $G/r06/c4_band_timer.txt $P/r06_c4_band_timer.txt
python3 scripts/summarize_prof.py $(find $G/r06/c4kt -name run_kernel_trace.csv) "C4 8K rgb8, 8 bands, 2 in flight, kernel records" > $P/r06_c4_kernel_trace.md
grep '^{' $G/r06/bench.json | tail -1 > $P/r06a_bench.json
grep -h -o '"src_sha256": "[0-9a-f]\{8\}' $P/pmc_lk_iter.json $P/pmc_step.json $P/pmc_warp_diff.json $P/warp_kernel_trace.json $P/warp_kernel_trace_projective.json | sort | uniq -c
