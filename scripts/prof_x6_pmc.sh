set -o pipefail
o=gpurun_out/x6pmc
scripts/prof_pmc.sh $o/p1 sgemm "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" --set variant=20 &&
scripts/prof_pmc.sh $o/p2 sgemm "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE" --set variant=20 &&
scripts/prof_pmc.sh $o/p3 sgemm "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" --set variant=20 &&
for p in p1 p2 p3; do echo "== $p"; python scripts/pmc_summary.py $(ls $o/$p/*counter_collection.csv | head -1) sgemm_x6; done > $o/summary.txt
