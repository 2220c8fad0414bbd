"""N <= 256 attention (k_attn_bf16_pipe): at its start every workgroup also touches the Q / K / V lines of the unit
PF_DIST blocks ahead (two global_load_dword per wave, one lane per 128-B line, results discarded), so that unit's loads,
a round of workgroups later, find its lines in the Infinity Cache instead of HBM and the HBM reads are spread over the
compute phases (round 6: the N sweep shows a large per-unit fixed cost, r6_lab/attn_nsweep.txt). The prefetches are
the youngest vector-memory ops of the wave at the counted waits (+2 each) and retired before the output stores."""
PF_DIST = 1024
_DMA_END = '''                                             (lptr_t)(img + g * 1024), 16, 0, 0);
        }
    }
'''
EDITS = [
    ("attention.hip", _DMA_END, _DMA_END + '''    int pf0, pf1;
    {
        // unit bh + PF_DIST (clamped into the grid): lines i = tid, tid + 512 of its 3 N rows (q, k, v of each token)
        const int pu = min(bh + PF_DIST, (int)gridDim.x - 1);
        const int pb = pu / H, ph = pu - (pu / H) * H;
        const bf16_t* pbase = qkv + (int64_t)pb * N * 3 * D + ph * HD;
        const int i0 = min(tid, 3 * N - 1), i1 = min(tid + 512, 3 * N - 1);
        const bf16_t* a0 = pbase + (int64_t)(i0 / 3) * 3 * D + (i0 % 3) * D;
        const bf16_t* a1 = pbase + (int64_t)(i1 / 3) * 3 * D + (i1 % 3) * D;
        asm volatile("global_load_dword %0, %1, off" : "=v"(pf0) : "v"(a0));
        asm volatile("global_load_dword %0, %1, off" : "=v"(pf1) : "v"(a1));
    }
'''),
    ("attention.hip", "    wait_vmcnt(NT);\n    asm volatile(\"\" : \"+v\"(qf[0]), \"+v\"(qf[1]), \"+v\"(qf[2]), \"+v\"(qf[3]) :: \"memory\");\n    const bool active = sid < nstrips;",
     "    wait_vmcnt(NT + 2);\n    asm volatile(\"\" : \"+v\"(qf[0]), \"+v\"(qf[1]), \"+v\"(qf[2]), \"+v\"(qf[3]) :: \"memory\");\n    const bool active = sid < nstrips;"),
    ("attention.hip", "                wait_vmcnt(max(NT - c - CPB, 0));", "                wait_vmcnt(max(NT - c - CPB, 0) + 2);"),
    ("attention.hip", "        run_strip(std::true_type{}, o0, o1, o16, m, l);\n",
     "        run_strip(std::true_type{}, o0, o1, o16, m, l);\n        asm volatile(\"s_waitcnt vmcnt(0)\" :: \"v\"(pf0), \"v\"(pf1) : \"memory\");\n"),
    ("attention.hip", "    run_strip(std::false_type{}, o0, o1, o16_unused, m, l);\n",
     "    run_strip(std::false_type{}, o0, o1, o16_unused, m, l);\n    asm volatile(\"s_waitcnt vmcnt(0)\" :: \"v\"(pf0), \"v\"(pf1) : \"memory\");\n"),
]
DEFINES = [f"-DPF_DIST={PF_DIST}"]
