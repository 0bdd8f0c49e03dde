set -u
mkdir -p gpurun_out/exp_c; export TMPDIR=/tmp
O=gpurun_out/exp_c
timeout -k 10 120 tools/valu_rate 4096 > $O/valu_rate.log 2>&1; echo "valu_rate rc=$?"; cat $O/valu_rate.log
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $O/valu_pmc -o run --output-format csv -- tools/valu_rate 65536 > $O/valu_pmc.log 2>&1; echo "valu pmc rc=$?"
R="python3 tools/render_once.py"
RT_LAUNCH_LOG=1 timeout -k 10 120 $R --config C3 --spp 16 > $O/c3_launch.log 2>&1; echo "c3 log rc=$?"; cat $O/c3_launch.log | head
timeout -k 10 300 $R --config C4 --spp 50 --reps 2 > $O/c4_base.log 2>&1; echo "c4 base rc=$?"; cat $O/c4_base.log
RT_TUNE=0x100000 timeout -k 10 300 $R --config C4 --spp 50 --reps 2 > $O/c4_pruneexp.log 2>&1; echo "c4 prune-exp rc=$?"; cat $O/c4_pruneexp.log
RT_TUNE=0x100002 timeout -k 10 300 $R --config C4 --spp 50 --reps 2 > $O/c4_pruneexp_noleaf.log 2>&1; echo "c4 prune-exp no-leaf rc=$?"; cat $O/c4_pruneexp_noleaf.log
RT_LAUNCH_LOG=1 timeout -k 10 300 $R --config C4 --reps 1 > $O/c4_full.log 2>&1; echo "c4 full rc=$?"; cat $O/c4_full.log
RT_SAMPLE_BUFFER_MB=8192 timeout -k 10 300 $R --config C4 --reps 1 > $O/c4_full_8g.log 2>&1; echo "c4 full 8G rc=$?"; cat $O/c4_full_8g.log
