# K-assembly counters for the headline's composed instance (SE+SE+WN: kmat_symu_kernel<2, 2>),
# instruction mix and busy cycles (two --pmc passes, <= 8 SQ counters each),
# a kernel trace, and the stores-compiled-out build's time.  Summarised by tools/kpmc_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kpmc6
O=gpurun_out/kpmc6
export KB_ONLY=SE+SE+WN
timeout -k 10 120 ./tools/kbuild_bench > $O/plain.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/kbuild_bench_nostore > $O/nostore.txt 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d $O/p1 -o p -- ./tools/kbuild_bench > $O/p1.txt 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p2 -o p -- ./tools/kbuild_bench > $O/p2.txt 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/p3 -o p -- ./tools/kbuild_bench > $O/p3.txt 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/tr -o p -- ./tools/kbuild_bench > $O/tr.txt 2>&1 || exit 6
echo done
