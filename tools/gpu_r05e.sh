# K-assembly PMC passes: instruction mix, busy cycles and HBM bytes of the
# kernel-matrix builds (tools/kbuild_bench, SE only: symmetric full, cross, upper-only), one
# --pmc pass per counter group; then a kernel-trace profile of the eigensolver at n = 4096
# beside rocSOLVER dsyevd (quadrature methods 1 and 2, syev with m = 3 and m = n).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kpmc
O=gpurun_out/kpmc
export KB_ONLY=SE
timeout -k 10 120 ./tools/kbuild_bench > $O/plain.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d $O/p1 -o p -- ./tools/kbuild_bench > $O/p1.txt 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p2 -o p -- ./tools/kbuild_bench > $O/p2.txt 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/p3 -o p -- ./tools/kbuild_bench > $O/p3.txt 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p4 -o p -- ./tools/kbuild_bench > $O/p4.txt 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/tr -o p -- ./tools/kbuild_bench > $O/tr.txt 2>&1 || exit 6
unset KB_ONLY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/eigprof -o eig -- python3 tools/tridiag_probe.py 4096 1,2 > gpurun_out/eigprof.txt 2>&1 || exit 7
echo done
