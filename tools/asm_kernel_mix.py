"""Instruction mix of one kernel in a `hipcc -S --cuda-device-only` listing
(tools only): python tools/asm_kernel_mix.py FILE.s NAME_SUBSTRING"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
i = m.start()
j = s.find(".Lfunc_end", i)
body = [ln.strip() for ln in s[i:j].split("\n") if ln.startswith("\t") and not ln.startswith("\t.") and not ln.startswith("\t;")]
print(m.group(1), "instructions", len(body))
for pat in ["s_load_dwordx16", "s_load_dwordx8", "s_load_dwordx4", "s_load_dwordx2", "s_load_dword ", "global_load", "global_store",
            "ds_read", "ds_write", "v_fma_f64", "v_mfma", "s_waitcnt", "v_readlane", "v_readfirstlane", "v_writelane",
            "v_accvgpr", "scratch_", "s_cbranch", "v_cndmask"]:
    print(f"  {pat:18s} {sum(1 for ln in body if ln.startswith(pat.strip()))}")
