// sc_model.hpp -- cascade model: libconfig-subset reader/writer and the
// typed cascade the detect path consumes.
//
// Mirrors the reference's Model::Load / Model::Save (ObjDetector/Model.cpp
// :97-194 / :21-95) and the libconfig 1.4.9 text format they go through
// (scanner tokens scanner.c:1111-1190, writer libconfig.c:168-243,631-653,
// typed access libconfigcpp.c++:700-716,1137-1145).  The library itself is
// not used; this is a self-contained reader for the subset Save emits plus
// the usual comment / separator forms.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace sc {

struct CfgValue {
    enum Type { Group, List, Array, Int, Int64, Float, Bool, String };
    Type type = Group;
    std::string name;  // empty for list/array elements
    int64_t ival = 0;
    double fval = 0.0;
    std::string sval;
    std::vector<CfgValue> items;

    const CfgValue *find(const std::string &key) const;
};

// Throws sc::Error with code SC_ERR_PARSE on syntax errors.
CfgValue cfg_parse(const std::string &text);
std::string cfg_write(const CfgValue &root);
std::string cfg_format_float(double v);

struct WeakLR {  // LogisticRegression + liblinear model fields (Model.cpp:154-180)
    int patch_index = 0;
    double eps = 0.01, C = 0.1;
    int nr_class = 2, nr_feature = 32;
    double bias = 1.0;
    std::vector<float> w;  // nr_feature + 1 = 33
    int label[2] = {1, -1};
};

struct Stage {  // StageClassifier + GentleAdaboost fields (Model.cpp:131-152)
    float search_step = 0.01f, auc_step = 0.05f, TPR_min = 0.995f;
    int n_total = 0, n_pos = 0, n_neg = 0;
    float FPR = 0, TPR = 0, theta = 0, total_AUC_score = 0;
    int sample_num = 960, max_iters = 100;
    std::vector<WeakLR> weak;
};

struct Cascade {  // CascadeClassifier fields (Model.cpp:124-129)
    int max_stages_num = 10;
    float FPR_target = 1e-6f, TPR_min_perstage = 0.995f, FPR = 0, TPR = 0;
    std::vector<Stage> stages;
    int total_weak() const;
};

struct Error {
    int code;
    std::string msg;
};

Cascade cascade_from_cfg(const CfgValue &root);  // strict Model::Load
CfgValue cascade_to_cfg(const Cascade &c);       // Model::Save tree
void validate_for_detect(const Cascade &c, int n_patches);

std::vector<int32_t> extract_patches(int tmpl_w, int tmpl_h);  // x,y,w,h

}  // namespace sc
