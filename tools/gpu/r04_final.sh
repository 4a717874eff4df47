set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04final; mkdir -p $O
bash tools/gpu/trace.sh $O/c2_trace || exit 1
bash tools/gpu/profile.sh $O/final_c2 hotpot90k || exit 1
bash tools/gpu/profile.sh $O/final_c3 synth5m || exit 1
