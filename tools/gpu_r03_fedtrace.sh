# Kernel + copy timelines of the host-fed MSM under several piece schedules.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for spec in ${FT_SPECS:-"SVGPU_H2D_PIECES=3" "SVGPU_H2D_PIECES=4" "SVGPU_H2D_SPLIT=2,3,3,3,3,1"}; do
  tag=$(echo "$spec" | tr '=,' '__')
  export ${spec}
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof/ft_$tag -o run -- python3 tools/host_path_trace.py > gpurun_out/prof/ft_$tag.log 2>&1 || { echo "trace $spec failed"; tail -5 gpurun_out/prof/ft_$tag.log; exit 1; }
  unset SVGPU_H2D_PIECES SVGPU_H2D_SPLIT
  python3 tools/trace_timeline.py gpurun_out/prof/ft_$tag -5 > gpurun_out/tl_arrays_$tag.txt
  python3 tools/trace_timeline.py gpurun_out/prof/ft_$tag -1 > gpurun_out/tl_refs_$tag.txt
  echo "$spec arrays $(tail -1 gpurun_out/tl_arrays_$tag.txt | awk '{print $2}') us, refs $(tail -1 gpurun_out/tl_refs_$tag.txt | awk '{print $2}') us"
done
