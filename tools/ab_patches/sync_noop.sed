# k_etsi_sync finds no bursts: no jobs, so no Viterbi work either (timing only)
/    __shared__ SyncLds L;/a\    if (C >= 0) return;   // timing variant
