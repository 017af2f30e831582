# banked decimator passes with 4 input batches in flight
s/^constexpr int SOS_PD = 2;/constexpr int SOS_PD = 4;/
