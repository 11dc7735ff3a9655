"""trivy_amd: MI355X-native drop-in for mmorel-35/trivy's secret-scanning path
(pkg/fanal/secret).  See DESIGN.md; the C-ABI is include/trivy_secret.h."""
from .secret import (ConfigError, GetBuiltinRules, NewScanner, ParseConfig,  # noqa: F401
                     ScanArgs, Scanner)
