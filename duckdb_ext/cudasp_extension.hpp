// DuckDB extension class for the MI355X cudasp_scan (same name and loader
// entry point as the reference, src/include/cudasp_extension.hpp:7-12).
#pragma once

#include "duckdb.hpp"

namespace duckdb {

class CudaspExtension : public Extension {
public:
	void Load(ExtensionLoader &loader) override;
	std::string Name() override;
	std::string Version() const override;
};

} // namespace duckdb
