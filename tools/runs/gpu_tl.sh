# kernel timeline of the multi-stream full path (rocprofv3 kernel trace)
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
V=${1:-"full path l2 inplace x4"}
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/tl" -o run --output-format csv -- python "$R0/tools/kbench.py" --streams 4 --rounds 1 --iters 40 --only "$V" > "$R0/gpurun_out/tl.log" 2>&1
rc=$?; grep median "$R0/gpurun_out/tl.log"; [ $rc -ne 0 ] && { tail -5 "$R0/gpurun_out/tl.log"; exit $rc; }
F=$(ls "$R0"/gpurun_out/tl/*kernel_trace.csv "$R0"/gpurun_out/tl/*/*kernel_trace.csv 2>/dev/null | head -1)
head -1 "$F"
python "$R0/tools/timeline.py" "$F" --last 48
