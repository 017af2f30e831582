# the trellis runs on rows left as they are: no descramble / block loads (timing only)
s|    if (act) {   // the quad loads the block's type-5 soft bits and scrambler bytes as dwords|    if (act \&\& nj < 0) {   // timing variant: gather skipped|
