{{/* Common labels used by selectors in .devspace/config.yaml */}}
{{- define "devspace.labels" -}}
app.kubernetes.io/name: {{ .root.Release.Name | quote }}
app.kubernetes.io/component: {{ .component.name | quote }}
app.kubernetes.io/managed-by: devspace
release: {{ .root.Release.Name | quote }}
{{- end -}}

{{/* Total amd.com/gpu requested by a component's containers */}}
{{- define "devspace.gpus" -}}
{{- $n := 0 -}}
{{- range $c := .containers -}}
{{- if $c.resources -}}{{- if $c.resources.limits -}}{{- if $c.resources.limits.gpu -}}
{{- $n = add $n $c.resources.limits.gpu -}}
{{- end -}}{{- end -}}{{- end -}}
{{- end -}}
{{- $n -}}
{{- end -}}
