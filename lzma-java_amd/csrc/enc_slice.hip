// enc_slice.hip -- the parser of enc.hip compiled once more for the sliced encode
// (lzma_enc_session_*, include/lzma_mi355x.h): a launch stops at the first CodeOneBlock
// boundary (Encoder.java:843-936, _additionalOffset == 0) past its stop position and saves
// the encoder's state to HBM, or resumes from that state. Kept out of the batch kernels, whose
// register allocation is tight: they are compiled without it (LZG_ENC_SLICED = 0).
#define LZG_ENC_SLICED 1
#include "enc.hip"
