"""A/B build variants of the HIP module (``python -m fast_tffm_amd.build_native --variant NAME``,
selected at run time with ``FM_HIP_VARIANT=NAME``): name -> extra hipcc flags.

Kept out of build_native.py because that file is part of every module's content hash: adding a
variant here leaves the other builds current (a variant's own flags are hashed into its build).
"""

HIP_VARIANTS: dict[str, list[str]] = {"fwdnopf": ["-DFM_FWD_PREFETCH=0"], "fwdgen": ["-DFM_FWD_SPECIALIZE=0"],
                                     "bwdgen": ["-DFM_BWD_SPECIALIZE=0"],
                                     "allgen": ["-DFM_FWD_SPECIALIZE=0", "-DFM_BWD_SPECIALIZE=0"],
                                     "fu10w4": ["-DFM_FWD_UNR16=10", "-DFM_FWD_LOCAL_W16=4"],
                                     "f4gen": ["-DFM_FWD_UNR4=0", "-DFM_FWD_LOCAL_W4=0"],
                                     "cu32_8": ["-DFM_CHUNK_UNR32=8"],
                                     "sh16u2w7": ["-DFM_FWD_UNR16_SH=2", "-DFM_FWD_SH_W16=7"],
                                     "sh16u4w6": ["-DFM_FWD_UNR16_SH=4", "-DFM_FWD_SH_W16=6"],
                                     "sh16u6w5": ["-DFM_FWD_UNR16_SH=6", "-DFM_FWD_SH_W16=5"],
                                     "mfma": ["-DFM_WITH_MFMA=1"], "mfprof": ["-DFM_WITH_MFMA=1", "-DFM_MF_PROF=1"],
                                     "fp8slow": ["-DFM_FP8_FAST_EPI=0"], "r1nomask": ["-DFM_R1_MASK=0"],
                                     "chunkperm": ["-DFM_CHUNK_PERM=1"], "fp8narrow": ["-DFM_FP8_WIDE=0"],
                                     "fp8narrowapply": ["-DFM_FP8_WIDE_APPLY=0"],
                                     "fp8narrowcomb": ["-DFM_FP8_WIDE_COMBINE=0"],
                                     "nopin": ["-DFM_FMA_PIN=0"]}
