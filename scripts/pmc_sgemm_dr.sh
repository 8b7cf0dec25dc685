# Two PMC passes (kernel trace + counters only) over the SGEMM kernels named in $1 (default prod,34,torch).
set -e
export TMPDIR=/tmp
V=${1:-prod,34,torch}
O=gpurun_out/sgdr_pmc
mkdir -p $O
python3 -c "import sys; sys.path.insert(0,'scripts'); import _lab; _lab.lab_lib('sgemm_dr_lab','pcmx_sgemm_dr_lab_variant')"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o p -- python3 scripts/sgemm_dr_pmc.py 8192 $V > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU -d $O/p2 -o p -- python3 scripts/sgemm_dr_pmc.py 8192 $V > $O/p2.log 2>&1
for p in p1 p2; do f=$(find $O/$p -name "*counter_collection.csv" | head -1); for k in sgemm_rs sgemm_drp sgemm_dr_ Cijk; do echo "== $p $k"; python3 scripts/pmc_summary.py $f $k; done; done > $O/summary.txt
cat $O/summary.txt
