"""Counter groups for tools/pmc_gemm.sh: the wanted counters that this box's `rocprofv3 -L` lists, packed into passes
that respect the per-block limits (<= 8 SQ, 4 TCP, 2 TA, 2 TD, 2 GRBM; TCC / FETCH_SIZE kept out: the traffic passes
are tools/gpu_session.sh pmc). Prints name:ctr1,ctr2,... per pass."""
import re
import sys

text = open(sys.argv[1]).read()
avail = set(re.findall(r"\b([A-Z][A-Z0-9_]+(?:_sum|_avr|_max|_min)?)\b", text))
want = {
    "sq_time": ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    "sq_mem": ["SQ_INSTS_VMEM", "SQ_ACTIVE_INST_VMEM", "SQ_INST_LEVEL_VMEM", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
               "SQ_INSTS_LDS", "SQ_ACTIVE_INST_MISC", "GRBM_COUNT"],
    "sq_issue": ["SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA", "SQ_INST_CYCLES_VMEM", "SQ_ACTIVE_INST_SCA",
                 "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "GRBM_GUI_ACTIVE"],
    "ta": ["TA_BUSY_avr", "TA_TA_BUSY_sum", "GRBM_GUI_ACTIVE"],
    "ta2": ["TA_BUFFER_READ_WAVEFRONTS_sum", "TA_FLAT_READ_WAVEFRONTS_sum", "GRBM_GUI_ACTIVE"],
    "td": ["TD_TD_BUSY_sum", "TD_BUSY_avr", "GRBM_GUI_ACTIVE"],
    "tcp": ["TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCC_READ_REQ_LATENCY_sum",
            "TCP_TCC_READ_REQ_sum", "GRBM_GUI_ACTIVE"],
}
limits = {"SQ": 8, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2}
for name, ctrs in want.items():
    use, used = [], {}
    for c in ctrs:
        if c not in avail and c.rsplit("_", 1)[0] not in avail:
            continue
        blk = c.split("_", 1)[0]
        if used.get(blk, 0) >= limits.get(blk, 0):
            continue
        used[blk] = used.get(blk, 0) + 1
        use.append(c)
    if use:
        print(f"{name}:{','.join(use)}")
