"""The image path around the secret scanner, host side:

  Artifact.inspect        pkg/fanal/artifact/image/image.go:322-345 -- layers
                          whose diff ID is a base layer are analysed with the
                          secret analyzer disabled (:331-335)
  guessBaseLayers         image.go:526-554 + pkg/fanal/image/image.go:111-137
  inspectLayer / Walk     walker.LayerTar.Walk + AnalyzeFile per layer
                          (tsg_scan_layer_stream)
  image-config secrets    pkg/fanal/analyzer/imgconf/secret/secret.go:39-62
                          (json.MarshalIndent(config) scanned as config.json)
  ApplyLayers + report    applier/docker.go:297-316, scanner/local/scan.go:
                          236-254,487-496, report/json.go:22-50 (tsg_report_json)

Every layer is streamed (tsg_scan_layer_stream: the tar read in order, its
kept files scanned on the HIP path in bounded batches while the rest is read),
and the layers run concurrently on the one engine, as inspect's
parallel.NewPipeline does (image.go:327, --parallel workers, default 5); the
report bytes come from the C result objects."""
import io
from concurrent.futures import ThreadPoolExecutor

from . import report as R
from . import secret as S


def ScanImage(scanner, layers, config_json, diff_ids, layer_refs=None, artifact_name="", created_at=None,
              skip_files=(), skip_dirs=(), severities=None, threads=0, parallel=5, batch_bytes=0):
    """layers: uncompressed layer tars in image order -- bytes, or binary file
    objects read in order (an io.Reader each) -- diff_ids the matching rootfs
    diff IDs.  Returns (report bytes, per-layer types.Secret lists, base diff
    IDs)."""
    if len(layers) != len(diff_ids):
        raise ValueError("one diff ID per layer")
    base = set(R.GuessBaseLayers(config_json, diff_ids)) if config_json else set()

    def inspect_layer(item):
        tar, did = item
        if did in base:                  # secret analyzer disabled for base layers (image.go:331-335)
            return R.ScanResult.from_secrets([])
        reader = io.BytesIO(tar) if isinstance(tar, (bytes, bytearray, memoryview)) else tar
        res, _walk = S.ScanLayerStream(scanner, reader, skip_files=skip_files, skip_dirs=skip_dirs, threads=threads,
                                       batch_bytes=batch_bytes, as_result=True)
        return res
    with ThreadPoolExecutor(max_workers=max(1, parallel)) as ex:   # parallel.NewPipeline(workers, ...)
        results = list(ex.map(inspect_layer, zip(layers, diff_ids)))
    secrets = [res.secrets() for res in results]
    cfg_res = None
    if config_json:
        cfg_res = scanner.ScanBatchResult([S.ScanArgs("config.json", R.ImageConfigContent(config_json))])
    refs = layer_refs if layer_refs is not None else [{"DiffID": d} for d in diff_ids]
    kw = {} if created_at is None else {"created_at": created_at}
    doc = R.JSONReport(results, layer_refs=refs, image_config=cfg_res, artifact_name=artifact_name,
                       artifact_type="container_image", severities=severities, **kw)
    return doc, secrets, sorted(base, key=diff_ids.index)
