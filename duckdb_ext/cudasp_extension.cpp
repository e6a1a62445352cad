// DuckDB glue for the MI355X cudasp_scan (written against the DuckDB 1.4.x
// C++ extension API the reference targets, .github/workflows/MainDistributionPipeline.yml:19).
//
// Registers the same table in-out function as the reference
// (src/cudasp_extension.cu:626-635) and maps each DuckDB callback 1:1 onto the
// DuckDB-free host of include/cudasp_host.h, which runs the kernels of
// include/cudasp_abi.h.  All state-machine logic (validation, accumulation,
// batching, round-robin GPU, emit) lives in the host library so that it is
// tested without DuckDB (tests/test_host_bind.py, tests/test_sql_cases_gpu.py).
//
// Not compiled in this repository's CI: DuckDB's headers are not available in
// the build image.  Build recipe: INTEGRATION.md.
#define DUCKDB_EXTENSION_MAIN
#include "cudasp_extension.hpp"

#include <cstdlib>
#include <thread>

#include "duckdb.hpp"
#include "duckdb/common/exception.hpp"
#include "duckdb/function/table_function.hpp"

#include "cudasp_abi.h"
#include "cudasp_host.h"

namespace duckdb {

struct CudaspScanBindData : public TableFunctionData {
	cudasp_tf_bind_data *handle = nullptr;
	bool full_x = false; // outputs column is BLOB[] of x-only keys
	~CudaspScanBindData() override {
		cudasp_tf_bind_free(handle);
	}
};

struct CudaspScanState : public GlobalTableFunctionState {
	cudasp_tf_global *handle = nullptr;
	~CudaspScanState() override {
		cudasp_tf_global_free(handle);
	}
	idx_t MaxThreads() const override {
		return 64;
	}
};

struct CudaspScanLocalState : public LocalTableFunctionState {
	cudasp_tf_local *handle = nullptr;
	~CudaspScanLocalState() override {
		cudasp_tf_local_free(handle);
	}
};

static cudasp_tf_blob_arg BlobArg(const Value &v) {
	cudasp_tf_blob_arg a {nullptr, 0, 0};
	if (v.type().id() == LogicalTypeId::BLOB && !v.IsNull()) {
		auto &s = StringValue::Get(v);
		a.data = reinterpret_cast<const uint8_t *>(s.data());
		a.size = s.size();
		a.is_blob = 1;
	}
	return a;
}

static unique_ptr<FunctionData> CudaspScanBind(ClientContext &context, TableFunctionBindInput &input,
                                               vector<LogicalType> &return_types, vector<string> &names) {
	uint32_t argc = static_cast<uint32_t>(input.inputs.size());
	cudasp_tf_blob_arg scan {nullptr, 0, 0}, spend {nullptr, 0, 0};
	int labels_is_list = 0;
	vector<cudasp_tf_blob_arg> labels;
	if (argc == 4) {
		scan = BlobArg(input.inputs[1]);
		spend = BlobArg(input.inputs[2]);
		auto &lv = input.inputs[3];
		if (lv.type().id() == LogicalTypeId::LIST) {
			labels_is_list = 1;
			for (auto &child : ListValue::GetChildren(lv)) {
				labels.push_back(BlobArg(child));
			}
		}
	}
	int has_bs = 0, bs_int = 0;
	int64_t bs = 0;
	auto entry = input.named_parameters.find("batch_size");
	if (entry != input.named_parameters.end()) {
		has_bs = 1;
		auto tid = entry->second.type().id();
		if (tid == LogicalTypeId::INTEGER || tid == LogicalTypeId::BIGINT) {
			bs_int = 1;
			bs = entry->second.GetValue<int64_t>();
		}
	}
	auto result = make_uniq<CudaspScanBindData>();
	char err[512];
	if (cudasp_tf_bind(argc, scan, spend, labels_is_list, labels.data(), static_cast<uint32_t>(labels.size()),
	                   has_bs, bs_int, bs, &result->handle, err, sizeof(err)) != 0) {
		throw InvalidInputException(err);
	}
	// Protocol variants: output_count := INTEGER,
	// label_negation := BOOLEAN, full_x := BOOLEAN.
	auto param = [&](const char *name, int &has, int64_t &v) {
		auto it = input.named_parameters.find(name);
		has = it != input.named_parameters.end() && !it->second.IsNull();
		v = has ? it->second.GetValue<int64_t>() : 0;
	};
	int has_k, has_neg, has_fx;
	int64_t k, neg, fx;
	param("output_count", has_k, k);
	param("label_negation", has_neg, neg);
	param("full_x", has_fx, fx);
	if (cudasp_tf_bind_options(result->handle, has_k, k, has_neg, neg != 0, has_fx, fx != 0, err, sizeof(err)) != 0) {
		throw InvalidInputException(err);
	}
	result->full_x = has_fx && fx != 0;
	return_types = {LogicalType::BLOB, LogicalType::INTEGER, LogicalType::BLOB};
	names = {"txid", "height", "tweak_key"};
	return std::move(result);
}

static unique_ptr<GlobalTableFunctionState> CudaspScanInit(ClientContext &context, TableFunctionInitInput &input) {
	auto &bind = input.bind_data->Cast<CudaspScanBindData>();
	auto state = make_uniq<CudaspScanState>();
	if (cudasp_tf_init(bind.handle, &state->handle) != 0) {
		throw IOException("cudasp_scan: %s", cudasp_last_error());
	}
	return std::move(state);
}

static unique_ptr<LocalTableFunctionState> CudaspScanLocalInit(ExecutionContext &context, TableFunctionInitInput &input,
                                                               GlobalTableFunctionState *global_state) {
	auto &g = global_state->Cast<CudaspScanState>();
	auto local = make_uniq<CudaspScanLocalState>();
	if (cudasp_tf_local_init(g.handle, &local->handle) != 0) {
		throw IOException("cudasp_scan: %s", cudasp_last_error());
	}
	return std::move(local);
}

static OperatorResultType CudaspScanFunction(ExecutionContext &context, TableFunctionInput &data, DataChunk &input,
                                             DataChunk &output) {
	auto &bind = data.bind_data->Cast<CudaspScanBindData>();
	auto &g = data.global_state->Cast<CudaspScanState>();
	auto &l = data.local_state->Cast<CudaspScanLocalState>();
	idx_t count = input.size();
	if (count == 0) {
		return OperatorResultType::NEED_MORE_INPUT;
	}
	// Columns by position: txid, height, tweak_key, outputs (src/cudasp_extension.cu:159-163),
	// handed over as DuckDB holds them (cudasp_tf_vectors): each vector's data,
	// selection and validity words, the list child over its list size.  No
	// per-row loop and no allocation here; the host copies the rows straight
	// into its batch slots (the reference re-reads every row into two heap
	// strings, :188-223).
	UnifiedVectorFormat txid, height, tweak, outs, child_fmt;
	input.data[0].ToUnifiedFormat(count, txid);
	input.data[1].ToUnifiedFormat(count, height);
	input.data[2].ToUnifiedFormat(count, tweak);
	input.data[3].ToUnifiedFormat(count, outs);
	auto &child = ListVector::GetEntry(input.data[3]);
	child.ToUnifiedFormat(ListVector::GetListSize(input.data[3]), child_fmt);
	auto vec = [](const UnifiedVectorFormat &f) {
		cudasp_tf_vector v;
		v.data = f.data;
		v.sel = f.sel->data();
		v.validity = f.validity.GetData();
		return v;
	};
	// BIGINT[] values, or with full_x BLOB[] x-only keys (string_t): the host
	// reads the child per the bind's full_x
	static_assert(sizeof(string_t) == sizeof(cudasp_tf_string), "string_t layout");
	static_assert(sizeof(list_entry_t) == sizeof(cudasp_tf_list_entry), "list_entry_t layout");
	cudasp_tf_vectors c {};
	c.count = static_cast<uint32_t>(count);
	c.txid = vec(txid);
	c.height = vec(height);
	c.tweak = vec(tweak);
	c.outputs = vec(outs);
	c.child = vec(child_fmt);
	if (cudasp_tf_function_vectors(bind.handle, g.handle, l.handle, &c) < 0) {
		throw IOException("cudasp_scan: %s", cudasp_last_error());
	}
	return OperatorResultType::NEED_MORE_INPUT;
}

static OperatorFinalizeResultType CudaspScanFinalFunction(ExecutionContext &context, TableFunctionInput &data,
                                                          DataChunk &output) {
	auto &bind = data.bind_data->Cast<CudaspScanBindData>();
	auto &g = data.global_state->Cast<CudaspScanState>();
	auto &l = data.local_state->Cast<CudaspScanLocalState>();
	auto out = make_uniq<cudasp_tf_output>();
	int rc = cudasp_tf_final(bind.handle, g.handle, l.handle, out.get());
	if (rc < 0) {
		throw IOException("cudasp_scan: %s", cudasp_last_error());
	}
	auto txid_data = FlatVector::GetData<string_t>(output.data[0]);
	auto height_data = FlatVector::GetData<int32_t>(output.data[1]);
	auto tweak_data = FlatVector::GetData<string_t>(output.data[2]);
	for (idx_t i = 0; i < out->count; i++) {
		txid_data[i] = StringVector::AddStringOrBlob(
		    output.data[0], string_t(reinterpret_cast<const char *>(out->txid_data[i]), out->txid_size[i]));
		height_data[i] = out->height[i];
		tweak_data[i] = StringVector::AddStringOrBlob(
		    output.data[2], string_t(reinterpret_cast<const char *>(out->tweak_data[i]), out->tweak_size[i]));
	}
	output.SetCardinality(out->count);
	return rc == CUDASP_TF_HAVE_MORE_OUTPUT ? OperatorFinalizeResultType::HAVE_MORE_OUTPUT
	                                        : OperatorFinalizeResultType::FINISHED;
}

static void LoadInternal(ExtensionLoader &loader) {
	// No process settings are needed: the host's device feeds size their
	// streams from the hardware queues the HIP runtime gives the process
	// (GPU_MAX_HW_QUEUES, 4 by default).
	// Cold start: build every GPU's fixed-base table and park a ready feed per
	// GPU in the background, so the session's first cudasp_scan only rebinds
	// its keys (a query that arrives earlier waits for, or shares, the same
	// once-per-device work).  CUDASP_PREWARM=0 turns it off.
	const char *pw = std::getenv("CUDASP_PREWARM");
	if (!(pw && std::atoi(pw) == 0)) {
		std::thread([] { (void)cudasp_tf_prewarm(0, nullptr); }).detach();
	}
	TableFunction func("cudasp_scan",
	                   {LogicalType::TABLE, LogicalType::BLOB, LogicalType::BLOB, LogicalType::LIST(LogicalType::BLOB)},
	                   nullptr, CudaspScanBind, CudaspScanInit, CudaspScanLocalInit);
	func.in_out_function = CudaspScanFunction;
	func.in_out_function_final = CudaspScanFinalFunction;
	func.named_parameters["batch_size"] = LogicalType::INTEGER;
	func.named_parameters["output_count"] = LogicalType::INTEGER;
	func.named_parameters["label_negation"] = LogicalType::BOOLEAN;
	func.named_parameters["full_x"] = LogicalType::BOOLEAN;
	loader.RegisterFunction(func);
}

void CudaspExtension::Load(ExtensionLoader &loader) {
	LoadInternal(loader);
}

std::string CudaspExtension::Name() {
	return "cudasp";
}

std::string CudaspExtension::Version() const {
	return cudasp_version();
}

} // namespace duckdb

extern "C" {
DUCKDB_CPP_EXTENSION_ENTRY(cudasp, loader) {
	duckdb::LoadInternal(loader);
}
}
