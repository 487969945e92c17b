// hpe_prog.h — word layout of a compiled "row program" (shared by hpe/compiler.py and the kernels).
//
// A head model of the reference (every builder in Model-96/train_96.py:65-110,
// Model-88/train_88.py:66-253, Model-88/attention_model.py:16-169 and all 684 checkpoint graphs) is,
// per spatial position, a DAG of 1x1-conv / dense GEMMs, element-wise epilogues and row-local
// normalisations.  The compiler lowers it to a flat op list that one persistent HIP kernel
// interprets over tiles of T rows held in LDS: activations never leave the CU, only the input
// rows stream from HBM.
#pragma once

#define HPE_MAGIC 0x31455048  // "HPE1"

// ---- header words ------------------------------------------------------------------------------
enum {
  H_MAGIC = 0, H_NOPS, H_NSLOTS, H_T, H_NW, H_IN_SLOT, H_OUT_SLOT, H_CIN, H_COUT,
  H_NPARAMS, H_NPARAMS_TRAIN, H_LDS_FLOATS, H_MAXACC, H_MAXTHIN, H_NTACC, H_OPS_OFF,
  H_SLOTS_OFF, H_BLK_OFF, H_TACC_OFF, H_MODE, H_WG_PER_CU, H_SCRATCH_OFF, H_NTHIN, H_SLAB,
  H_KIND,  // KIND_GENERIC: op list for rowprog_kernel; KIND_MLP2: one OP_MLP2 op for mlp2_kernel
  H_NPASS,   // generic training programs: launches per step, each owning NW * MAXACC dW blocks (0/1: one)
  H_GSLOTS,  // generic programs: 1 = tile slots in a per-workgroup device scratch region (too big for LDS)
  H_WORDS = 32
};

enum { MODE_FWD = 0, MODE_TRAIN = 1, MODE_EVAL = 2 };
enum { KIND_GENERIC = 0, KIND_MLP2 = 1, KIND_CHAIN = 2, KIND_RES = 3 };

// ---- slot words: LDS float offset, channels, padded channels (even, %8), row stride -----------
enum { S_OFF = 0, S_C, S_CP, S_STRIDE, S_WORDS = 4 };

// ---- op words -----------------------------------------------------------------------------------
enum {
  O_TYPE = 0, O_A, O_B, O_OUT, O_K, O_N, O_W, O_BIAS, O_FLAGS,
  O_EACT, O_EDROP, O_ETHR, O_EKEEP, O_EZ,   // epilogue: activation, dropout ordinal/threshold/keep-prob, z slot
  O_AUX0, O_AUX1, O_AUX2, O_AUX3, O_TBASE, O_TCOUNT, O_F0, O_F1, O_MODE, O_WSEL,
  O_WORDS = 24
};

enum {
  OP_DENSE = 1,    // out = epi(a . W + b)                       MFMA 32x32x2 f32
  OP_TDENSE = 2,   // same, N <= 8, VALU with K split over threads
  OP_EW = 3,       // out = epi((f0 a + f1 b | a * b) * s + t)
  OP_LN = 4,       // out = epi(LayerNorm(a))  (+ xhat / rstd for backward)
  OP_LOSS = 5,     // MSE/MAE partial sums; out = dL/dpred through the producer's epilogue
  OP_EPIGRAD = 6,  // out <- out * epi'(a)                       (in place)
  OP_DW = 7,       // dW blocks += a^T . b                       MFMA, register accumulators
  OP_TACC = 8,     // thin per-thread accumulators (small dW, bias, per-channel scale grads)
  OP_DIN = 9,      // out (=|+=|epigrad) a . W^T                 MFMA
  OP_TDIN = 10,    // same, contraction N <= 8, VALU
  OP_EWB = 11,     // backward of OP_EW
  OP_LNB = 12,     // backward of OP_LN
  // fused 2-layer regressor (hpe_mlp2.hip): x (C_in) -> dense F (act1, dropout1) -> dense 3
  // (act2, dropout2).  Fields: O_K C_in, O_N F, O_AUX3 N2 (=3), O_W W1, O_BIAS b1, O_AUX0 W2,
  // O_AUX1 b2, O_E* layer-1 epilogue, O_AUX2 act2, O_TBASE drop2 id, O_TCOUNT drop2 threshold,
  // O_F0 keep2, O_FLAGS row blocks per wave per tile (RBW), O_MODE column blocks (= waves).
  OP_MLP2 = 13,
  // fused narrow chain forward (hpe_chain.hip): x -> dense F1 <= 32 -> [dense F2 <= 32] -> dense 3.
  // Fields: O_K C_in, O_N F1, O_AUX3 F2 (0 = none), O_W W1, O_BIAS b1, O_AUX0 W2, O_AUX1 b2,
  // O_AUX2 W3, O_TBASE b3, O_EACT act1, O_FLAGS act2, O_MODE act3, O_TCOUNT 3.
  OP_CHAIN = 14,
  // fused residual stack (hpe_res.hip, training): x (C_in 88 | 96) -> dense 16 -> NB x [dense 16 ->
  // dense 16 -> add(block input) -> act] -> [dense BOT <= 16] -> dense 3 (create_model_complex,
  // Model-88/attention_model.py:97-169).  Fields: O_K C_in, O_N 16, O_AUX3 NB, O_FLAGS BOT (0 =
  // none), O_MODE the post-add activation, O_AUX0 word offset of the layer table, O_AUX1 its
  // entries (dense layers in order: 1 + 2 NB + [1] + 1), RL_WORDS each.
  OP_RES = 15
};
// residual-stack layer table entry: kernel / bias parameter offsets (-1: none), activation,
// dropout ordinal (-1: none), keep threshold, keep probability (float bits), K, N
enum { RL_W = 0, RL_B, RL_ACT, RL_DROP, RL_THR, RL_KEEP, RL_K, RL_N, RL_WORDS = 8 };

enum { EW_HAS_B = 1, EW_MUL = 2, EW_AFFINE = 4 };             // OP_EW / OP_EWB flags
enum { DST_STORE = 0, DST_ACCUM = 1, DST_EPIGRAD = 2 };       // O_MODE of DIN/TDIN/EWB/LNB
enum { TACC_GEMM = 0, TACC_BIAS = 1, TACC_DIAG = 2 };         // O_AUX3 of OP_TACC

enum {
  ACT_LINEAR = 0, ACT_TANH, ACT_RELU, ACT_SOFTSIGN, ACT_SIGMOID, ACT_ELU, ACT_SELU, ACT_SWISH,
  ACT_SOFTPLUS, ACT_LEAKY_RELU
};

// ------------------------------------------------------------------------------------------------
// BlazeFace backbone plan (csrc/hpe_blaze.hip; built by hpe/blazeface.py from the unified model's
// model_config).  Header of BFH_WORDS, then n_ops ops of BFO_WORDS.  Activations between ops are
// NHWC fp32 with the channel stride padded to a multiple of 8 (pad channels hold zeros).
// ------------------------------------------------------------------------------------------------
#define HPE_BF_MAGIC 0x46425048  // "HPBF"
enum { BFH_MAGIC = 0, BFH_NOPS, BFH_ACT_FLOATS, BFH_OPS_OFF, BFH_WORDS = 8 };
// BF_ROWS: a depthwise block streamed down the image in steps of TH output rows (ring of ROWS
// input rows in LDS, next step's rows prefetched into registers); BFO_NI = row segments per image
// BF_DIRECT: persistent, taps read from global, all output chunks per task (16x16 / 8x8 maps, heads)
// BF_STAGE: an execution record: the BFO_NI records after it (dw blocks on maps of <= 256
// positions, and the detector heads right after the block producing their tap) run as ONE launch,
// one workgroup per image, the map resident in LDS (bf_stage_kernel); BFO_CS = the map's channel
// stride, BFO_ROWS / BFO_COLS = floats of the map / W^T regions, BFO_LDS = bytes.  The covered
// records keep their per-op meaning (a reader that skips BF_STAGE computes the same outputs).
// BF_FRONT: an execution record: the BFO_NI = 6 records after it (the stem and the five blocks on the
// 64x64 / 32x32 maps of the BlazeFace backbone, BF_STEM + BF_ROWS records) run as ONE launch,
// one workgroup per frame, the maps streamed row by row through LDS rings (bf_front_kernel); only
// the frame and the last block's 32x32 output touch HBM.  BFO_LDS = bytes.
enum { BF_STEM = 1, BF_BLOCK = 2, BF_ROWS = 3, BF_DIRECT = 4, BF_STAGE = 5, BF_FRONT = 6 };
enum { BF_RES_NONE = 0, BF_RES_ID = 1, BF_RES_MAXPOOL = 2 };
// buffers: image input, two ping-pong activations, then the six caller outputs
enum { BF_BUF_IMG = 0, BF_BUF_A = 1, BF_BUF_B = 2, BF_BUF_OUT0 = 3, BF_NBUF = 9 };
enum {
  BFO_KIND = 0, BFO_H, BFO_W, BFO_HO, BFO_WO, BFO_CIN, BFO_COUT, BFO_CINP, BFO_COUTP,
  BFO_STRIDE, BFO_PADT, BFO_PADL, BFO_DW, BFO_RES, BFO_RELU, BFO_SRC, BFO_DST, BFO_DST2,
  BFO_SPLIT, BFO_TH, BFO_NI, BFO_DWW, BFO_PWW, BFO_PWB, BFO_CS, BFO_KS, BFO_ROWS, BFO_COLS,
  BFO_NC, BFO_LDS, BFO_OSTRIDE, BFO_NCT, BFO_WAVES, BFO_WORDS = 40
};
