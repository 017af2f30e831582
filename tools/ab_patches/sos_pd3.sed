# banked decimator passes with 3 input batches in flight
s/^constexpr int SOS_PD = 2;/constexpr int SOS_PD = 3;/
