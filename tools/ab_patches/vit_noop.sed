# k_etsi_viterbi returns at once: the lower MAC without its trellis (timing only)
/__shared__ __attribute__((aligned(16))) int8_t rows\[16 \* VROW\];/a\    if (kmask >= 0) return;   // timing variant
