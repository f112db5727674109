"""Cloud provider commands against a fake GraphQL provider (no network): add provider, login,
create/list/use/remove space, kube-context management, deploy into a space, reset."""

import json
import os

import yaml

from fake_cloud import FakeCloud, make_token


def test_cloud_space_lifecycle(localkube):
    lk = localkube
    cloud = FakeCloud(lk.cluster.server).start()
    try:
        proj = lk.project("quickstart", "quickstart-cloud")
        cfg_path = os.path.join(proj, ".devspace", "config.yaml")
        cfg = yaml.safe_load(open(cfg_path))
        cfg["cluster"] = {"cloudProvider": "fake"}
        open(cfg_path, "w").write(yaml.safe_dump(cfg))

        lk.run(["add", "provider", cloud.url, "--name", "fake"], proj)
        providers = yaml.safe_load(open(os.path.join(lk.home, ".devspace", "clouds.yaml")))
        assert providers["fake"]["host"] == cloud.url

        token = make_token("alice")
        out = lk.run(["login", "--provider", "fake", "--token", token], proj).stdout
        assert "Successful logged into fake" in out
        docker_cfg = json.load(open(os.path.join(lk.home, ".docker", "config.json")))
        assert "registry.fake.cloud" in json.dumps(docker_cfg)

        p = lk.run(["deploy"], proj, check=False)
        assert p.returncode != 0 and "No space configured" in p.stdout + p.stderr

        out = lk.run(["create", "space", "dev1"], proj).stdout
        assert "Successfully created space dev1" in out
        kc = yaml.safe_load(open(lk.kubeconfig))
        assert kc["current-context"] == "devspace-dev1"
        ctx = [c for c in kc["contexts"] if c["name"] == "devspace-dev1"][0]["context"]
        assert ctx["namespace"] == "space-dev1"
        gen = yaml.safe_load(open(os.path.join(proj, ".devspace", "generated.yaml")))
        assert gen["space"]["name"] == "dev1"

        assert "dev1" in lk.run(["list", "spaces"], proj).stdout

        out = lk.run(["deploy"], proj).stdout
        assert "Using space dev1" in out
        assert "https://dev1.fake.cloud" in out
        assert lk.pods("space-dev1"), "pods were not deployed into the space namespace"
        lk.run(["purge"], proj)

        lk.run(["use", "space", "none"], proj)
        gen = yaml.safe_load(open(os.path.join(proj, ".devspace", "generated.yaml")))
        assert not gen.get("space")
        lk.run(["use", "space", "dev1", "--context=false"], proj)
        lk.run(["use", "context", "dev1"], proj)
        kc = yaml.safe_load(open(lk.kubeconfig))
        assert kc["current-context"] == "devspace-dev1"
        out = lk.run(["remove", "context", "dev1"], proj).stdout
        assert "Successfully deleted kubectl context for space dev1" in out
        kc = yaml.safe_load(open(lk.kubeconfig))
        assert all(c["name"] != "devspace-dev1" for c in kc.get("contexts") or [])
        lk.run(["use", "context"], proj)  # no arg: the space configured in generated.yaml
        kc = yaml.safe_load(open(lk.kubeconfig))
        assert kc["current-context"] == "devspace-dev1"

        # use registry: docker credentials for the provider's account (cmd/use/registry.go)
        out = lk.run(["use", "registry", "registry.other.cloud"], proj).stdout
        assert "Successfully logged into registry registry.other.cloud" in out
        auths = json.load(open(os.path.join(lk.home, ".docker", "config.json")))["auths"]
        assert "registry.other.cloud" in auths and auths["registry.other.cloud"].get("auth")

        lk.run(["remove", "space", "dev1"], proj)
        assert not cloud.spaces
        kc = yaml.safe_load(open(lk.kubeconfig))
        assert all(c["name"] != "devspace-dev1" for c in kc.get("contexts") or [])

        lk.run(["remove", "provider", "fake"], proj)
        providers = yaml.safe_load(open(os.path.join(lk.home, ".devspace", "clouds.yaml")))
        assert "fake" not in providers
        assert all(auth.startswith("Bearer ey") for auth, _ in cloud.requests)
    finally:
        # restore the cluster kubeconfig for other tests in the module
        lk.cluster.write_kubeconfig(lk.kubeconfig)
        cloud.stop()
