"""Group/version registration for ``apps.kubedl.io/v1alpha1``.

Reference: ``api/v1alpha1/groupversion_info.go:27-40`` (GroupVersion,
``KindCron``, SchemeBuilder/AddToScheme) and ``pkg/common/constants.go:19-25``
(label keys).  The "scheme" here is the kind <-> resource table the runtime
and the fake apiserver share (:mod:`cron_operator_amd.runtime.scheme`).
"""
from __future__ import annotations

from ..meta import GroupVersion, GroupVersionKind, GroupVersionResource

GROUP = "apps.kubedl.io"
VERSION = "v1alpha1"
GROUP_VERSION = GroupVersion(GROUP, VERSION)

KIND_CRON = "Cron"
KIND_CRON_LIST = "CronList"
RESOURCE_CRONS = "crons"
SINGULAR_CRON = "cron"

CRON_GVK = GroupVersionKind(GROUP, VERSION, KIND_CRON)
CRON_GVR = GroupVersionResource(GROUP, VERSION, RESOURCE_CRONS)

# pkg/common/constants.go
LABEL_PREFIX_KUBEDL = "kubedl.io"
LABEL_CRON_NAME = LABEL_PREFIX_KUBEDL + "/cron-name"
