// msv_kernel_part.hip -- one part of the variant family: compiled once per msv_variants_<k>.inc
// (csrc/Makefile: -DMSV_PART=k -DMSV_PART_INC="msv_variants_k.inc"), so the ~90 instantiations of
// msv_batch_kernel build in parallel; msv_kernel.hip concatenates the parts in order.
#include "msv_kernel_impl.h"

#define MSV_CAT(a, b) a##b
#define MSV_XCAT(a, b) MSV_CAT(a, b)

namespace msvk {

static const Variant kPart[] = {
#include MSV_PART_INC
};

const Variant* MSV_XCAT(variants_part_, MSV_PART)(int* count) {
    *count = static_cast<int>(sizeof(kPart) / sizeof(kPart[0]));
    return kPart;
}

}  // namespace msvk
