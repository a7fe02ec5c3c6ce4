// launch_cfg.h -- launch shapes shared by the kernels and the host (h264r_host.hip)
#pragma once

// consecutive 16-MB groups per workgroup (k_recon.hip): k_inter4 / k_inter4r (1: with
// more, loop-carried state spilled and config 3 lost 2 %, profiles/r03_h_inter_ab.txt; 2
// still costs config 3 4 % while config 4 gains 2 %, profiles/r03s2_s_ab.txt)
#ifndef H264R_INTER_GROUPS
#define H264R_INTER_GROUPS 1
#endif

// k_deblock2: MB rows per wave, walked in lock step one MB apart (k_deblock2.hip); the
// wave's 16 (picture, row) units cover 16 / H264R_DB2_BAND pictures
#ifndef H264R_DB2_BAND
#define H264R_DB2_BAND 4
#endif

// k_deblock2: lanes per (picture, MB row) unit (4 or 8); a wave holds 64 / H264R_DB2_LPU units
#ifndef H264R_DB2_LPU
#define H264R_DB2_LPU 8
#endif
