bash profiles/scripts/r05_e2e_trace.sh && bash profiles/scripts/r05_profA.sh
