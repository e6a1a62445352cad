// The bound arguments of one cudasp_scan call (include/cudasp_host.h,
// cudasp_tf_bind): shared by the table-function host (cudasp_host.cpp) and the
// pinned tables (pinned_table.cpp).  Mirrors CudaspScanBindData
// (src/cudasp_extension.cu:87-104).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/cudasp_abi.h"
#include "../../../include/cudasp_host.h"

struct cudasp_tf_bind_data {
  uint64_t batch_size = CUDASP_TF_DEFAULT_BATCH;
  cudasp_scan_options opt{1, 0, 0};  // named parameters output_count / label_negation / full_x
  std::string scan_private_key_data;
  std::string spend_public_key_data;
  std::vector<std::string> label_keys_data;
  std::string label_keys_flat;  // label_count x 64, back to back
};
