s/__launch_bounds__(A2_T, 5) void k_pfb_analysis2/__launch_bounds__(A2_T, 4) void k_pfb_analysis2/
