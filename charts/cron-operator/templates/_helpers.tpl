{{/* Chart name, overridable with .Values.nameOverride. */}}
{{- define "cronop.name" -}}
{{- .Values.nameOverride | default .Chart.Name | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{/* Fully qualified release name (63 chars max, DNS label). */}}
{{- define "cronop.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- $base := .Values.nameOverride | default .Chart.Name -}}
{{- if contains $base .Release.Name -}}
{{- .Release.Name | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name $base | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}
{{- end -}}

{{/* Labels used by selectors: must stay stable across upgrades. */}}
{{- define "cronop.selectorLabels" -}}
app.kubernetes.io/name: {{ include "cronop.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}

{{/* Labels on every object. */}}
{{- define "cronop.labels" -}}
{{ include "cronop.selectorLabels" . }}
app.kubernetes.io/part-of: cron-operator
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" }}
{{- if .Chart.AppVersion }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
{{- end }}
{{- end -}}

{{/* registry/repository:tag, tag defaulting to appVersion then version. */}}
{{- define "cronop.image" -}}
{{- $tag := .Values.image.tag | default .Chart.AppVersion | default .Chart.Version -}}
{{- printf "%s/%s:%s" .Values.image.registry .Values.image.repository $tag -}}
{{- end -}}

{{/* Global node selector overridden key-by-key by the chart's own. */}}
{{- define "cronop.nodeSelector" -}}
{{- $sel := mergeOverwrite (deepCopy (.Values.global.nodeSelector | default dict)) (.Values.nodeSelector | default dict) -}}
{{- if eq .Values.global.clusterProfile "Edge" -}}
{{- $_ := set $sel "alibabacloud.com/is-edge-worker" "false" -}}
{{- end -}}
{{- if $sel }}{{ toYaml $sel }}{{ end -}}
{{- end -}}

{{/* Global tolerations followed by the chart's own (plus the Edge addon toleration). */}}
{{- define "cronop.tolerations" -}}
{{- $tol := concat (.Values.global.tolerations | default list) (.Values.tolerations | default list) -}}
{{- if eq .Values.global.clusterProfile "Edge" -}}
{{- $tol = append $tol (dict "key" "node-role.alibabacloud.com/addon" "operator" "Exists" "effect" "NoSchedule") -}}
{{- end -}}
{{- if $tol }}{{ toYaml $tol }}{{ end -}}
{{- end -}}
