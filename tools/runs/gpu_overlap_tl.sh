# Kernel timeline of the 3-stream C2 path (classify + group) vs classify alone (rocprofv3 kernel trace)
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
for cfg in in_place,1,3 in_place,0,3 read_only,1,3; do
  tag=$(echo $cfg | tr ',' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/tl_$tag" -o run --output-format csv -- python "$R0/tools/overlap_probe.py" --steps 60 --warmup 20 --only $cfg > "$R0/gpurun_out/tl_$tag.log" 2>&1
  rc=$?; grep '^{' "$R0/gpurun_out/tl_$tag.log"; [ $rc -ne 0 ] && { tail -5 "$R0/gpurun_out/tl_$tag.log"; exit $rc; }
  F=$(ls "$R0"/gpurun_out/tl_$tag/*kernel_trace.csv "$R0"/gpurun_out/tl_$tag/*/*kernel_trace.csv 2>/dev/null | head -1)
  echo "== $cfg"
  python "$R0/tools/timeline.py" "$F" --last 30 > "$R0/gpurun_out/tl_$tag.txt"
  tail -45 "$R0/gpurun_out/tl_$tag.txt"
done
exit 0
