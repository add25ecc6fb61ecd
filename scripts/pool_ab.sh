for spec in "--pack fp8 --layers 8 --layer-mib 3072" "--pack fp8 --layers 8 --layer-mib 3072 --source-pool 2" "--layers 24 --layer-mib 1024" "--layers 24 --layer-mib 1024 --source-pool 2" "--pack fp8 --layers 20 --layer-mib 3072"; do
  tag=$(echo "$spec" | tr -c 'a-z0-9' '_')
  timeout -k 10 300 python bench.py $spec --steps 2 --warmup 1 > gpurun_out/pool/$tag.json 2> gpurun_out/pool/$tag.log || exit 1
  grep "step 1" gpurun_out/pool/$tag.log
done
