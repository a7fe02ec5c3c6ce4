// launch_cfg.h -- launch shapes shared by the kernels and the host (h264r_host.hip)
#pragma once

// consecutive 16-MB groups per workgroup (k_recon.hip): k_inter4 / k_inter4r (1: with
// more, loop-carried state spilled and config 3 lost 2 %, profiles/r03_h_inter_ab.txt),
// k_dbinfo
#ifndef H264R_INTER_GROUPS
#define H264R_INTER_GROUPS 1
#endif
#ifndef H264R_DBINFO_GROUPS
#define H264R_DBINFO_GROUPS 4
#endif
